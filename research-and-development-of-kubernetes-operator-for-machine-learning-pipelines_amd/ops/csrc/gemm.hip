// bf16 GEMM on MFMA for gfx950 (K1 prefill / K2 decode / K13 MoE grouped).
//
//   C[M, N] = A[M, K] . B[N, K]^T        (A: activations row-major, B: weights [out, in])
//
// Tiling: a workgroup owns a BM x BN output tile, K is walked in BK = 64 steps
// through a double-buffered, XOR-swizzled LDS image (16-B chunk c of row r at
// chunk c ^ (r & 7): the 16 rows a ds_read_b128 lane group reads land on 8
// different 16-B bank slots, cdna_hip_programming.md §5.5 T2).  Staging is
// register-based and split (T14): the next tile's global loads are issued
// before the current tile's MFMAs and written to LDS after them.
// Waves are arranged WM x WN; each wave owns (BM/WM) x (BN/WN) as a grid of
// 16x16 accumulators fed by v_mfma_f32_16x16x32_bf16.
//
// Decode (M <= 256) is weight-streaming: BM covers the whole batch so every
// weight byte is read from HBM once; when the N tiles cannot fill 256 CUs the
// K range is split over blockIdx.z and fp32 partial slabs are combined by a
// second (reduce) kernel that also applies the epilogue (launch-boundary
// reduce, cdna_hip_programming.md §5 "Projection GEMM at M = 256" item 2).
//
// Epilogues (applied from an fp32 LDS copy of the tile, 16-B coalesced stores):
//   EPI_NONE      C = bf16(acc)
//   EPI_SILU_MUL  B rows are gate/up interleaved in groups of 16
//                 ([g0..g15, u0..u15, g16..g31, u16..u31, ...]) so a tile holds
//                 matching gate and up columns: C[:, j] = silu(gate_j) * up_j
//                 (C has N/2 columns) — fuses K8 into the gate_up projection.
//
// Grouped mode (MoE K13): A rows are sorted by expert, offsets[e]..offsets[e+1]
// are expert e's rows, B = W[e] ([E, N, K]); blockIdx.y enumerates
// (expert, m-tile) pairs (a block past the last pair exits immediately).
#include "common.h"
#include "launch.h"

namespace mlop {

enum { EPI_NONE = 0, EPI_SILU_MUL = 1 };
constexpr int kBK = 64;

template <int BM, int BN, int WM, int WN, int EPI, bool GROUPED>
__global__ void __launch_bounds__(WM * WN * 64) gemm_kernel(
    const uint16_t* __restrict__ A, int lda, const uint16_t* __restrict__ B, int ldb,
    uint16_t* __restrict__ C, int ldc, float* __restrict__ ws, int M, int N, int K, int k_chunk,
    const int* __restrict__ offsets, int n_groups) {
  constexpr int T = WM * WN * 64;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int CH = (BM + BN) * (kBK / 8);  // 16-B chunks per stage
  static_assert(CH % T == 0, "stage chunks must divide the thread count");
  constexpr int CPT = CH / T;
  constexpr int STAGE = (BM + BN) * kBK;  // bf16 elements per stage
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int n0 = blockIdx.x * BN;
  int m0 = blockIdx.y * BM, m_end = M;
  const uint16_t* Bg = B;
  if constexpr (GROUPED) {
    // find (expert, m-tile) of this block
    int t = blockIdx.y, e = 0;
    for (; e < n_groups; ++e) {
      const int rows = offsets[e + 1] - offsets[e];
      const int tiles = (rows + BM - 1) / BM;
      if (t < tiles) break;
      t -= tiles;
    }
    if (e >= n_groups) return;
    m0 = offsets[e] + t * BM;
    m_end = offsets[e + 1];
    Bg = B + (size_t)e * N * ldb;
  }
  const int kz = blockIdx.z;
  const int kbeg = kz * k_chunk;
  const int kend = min(K, kbeg + k_chunk);
  const int nk = (kend - kbeg) / kBK;

  u32x4 stage[CPT];
  auto gload = [&](int k) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = tid + i * T;
      const int r = c >> 3, ch = c & 7;
      if (r < BM) {
        const int gr = min(m0 + r, m_end - 1);
        stage[i] = *reinterpret_cast<const u32x4*>(A + (size_t)gr * lda + k + ch * 8);
      } else {
        const int gn = min(n0 + r - BM, N - 1);
        stage[i] = *reinterpret_cast<const u32x4*>(Bg + (size_t)gn * ldb + k + ch * 8);
      }
    }
  };
  auto sstore = [&](int buf) {
    uint16_t* base = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = tid + i * T;
      const int r = c >> 3, ch = c & 7;
      *reinterpret_cast<u32x4*>(base + r * kBK + ((ch ^ (r & 7)) << 3)) = stage[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    gload(kbeg);
    sstore(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kbeg + (kt + 1) * kBK);
    const uint16_t* sA = smem + buf * STAGE;
    const uint16_t* sB = sA + BM * kBK;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk * 4 + (lane >> 4);
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * WTM + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(sA + r * kBK + ((ch ^ (r & 7)) << 3));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * WTN + j * 16 + (lane & 15);
        bfr[j] = *reinterpret_cast<const bf16x8*>(sB + r * kBK + ((ch ^ (r & 7)) << 3));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }

  const int rows_here = min(BM, m_end - m0);
  if (gridDim.z > 1) {
    // split-K: fp32 partial slab [kz][M][N] (plain stores; reduce kernel in the next launch)
    float* P = ws + (size_t)kz * M * N;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * WTN + j * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ml = wm * WTM + i * 16 + 4 * (lane >> 4) + r;
          if (ml < rows_here && n < N) P[(size_t)(m0 + ml) * N + n] = acc[i][j][r];
        }
      }
    return;
  }
  // epilogue through LDS: fp32 tile [BM][BN + 4]
  float* sC = reinterpret_cast<float*>(smem);
  constexpr int LDC = BN + 4;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = wn * WTN + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) sC[(wm * WTM + i * 16 + 4 * (lane >> 4) + r) * LDC + n] = acc[i][j][r];
    }
  __syncthreads();
  if constexpr (EPI == EPI_NONE) {
    constexpr int VPR = BN / 8;
    for (int v = tid; v < BM * VPR; v += T) {
      const int r = v / VPR, c = (v % VPR) * 8;
      if (r >= rows_here || n0 + c >= N) continue;
      const float* s = sC + r * LDC + c;
      u32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = pack2(s[2 * j], s[2 * j + 1]);
      *reinterpret_cast<u32x4*>(C + (size_t)(m0 + r) * ldc + n0 + c) = o;
    }
  } else {
    constexpr int OUTW = BN / 2, VPR = OUTW / 8;
    for (int v = tid; v < BM * VPR; v += T) {
      const int r = v / VPR, j0 = (v % VPR) * 8;
      const int gcol = (j0 / 16) * 32 + (j0 % 16);
      if (r >= rows_here || n0 + gcol >= N) continue;
      const float* g = sC + r * LDC + gcol;
      const float* u = g + 16;
      u32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        // HF order: silu in bf16, then the product
        const float g0 = bf2f(f2bf(g[2 * j])), g1 = bf2f(f2bf(g[2 * j + 1]));
        const float s0 = bf2f(f2bf(g0 / (1.f + __expf(-g0))));
        const float s1 = bf2f(f2bf(g1 / (1.f + __expf(-g1))));
        o[j] = pack2(s0 * bf2f(f2bf(u[2 * j])), s1 * bf2f(f2bf(u[2 * j + 1])));
      }
      *reinterpret_cast<u32x4*>(C + (size_t)(m0 + r) * ldc + n0 / 2 + j0) = o;
    }
  }
}

// sum the split-K slabs and apply the epilogue; one thread per 8 outputs
template <int EPI>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(uint16_t* __restrict__ C, int ldc,
                                                           const float* __restrict__ ws, int M,
                                                           int N, int splits) {
  const int outw = EPI == EPI_NONE ? N : N / 2;
  const int vpr = outw / 8;
  const long total = (long)M * vpr;
  for (long v = blockIdx.x * (long)blockDim.x + threadIdx.x; v < total;
       v += (long)gridDim.x * blockDim.x) {
    const int r = (int)(v / vpr), j0 = (int)(v % vpr) * 8;
    const int col = EPI == EPI_NONE ? j0 : (j0 / 16) * 32 + (j0 % 16);
    float a[8] = {0, 0, 0, 0, 0, 0, 0, 0}, b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int s = 0; s < splits; ++s) {
      const float4* p = reinterpret_cast<const float4*>(ws + ((size_t)s * M + r) * N + col);
      float4 x = p[0], y = p[1];
      a[0] += x.x; a[1] += x.y; a[2] += x.z; a[3] += x.w;
      a[4] += y.x; a[5] += y.y; a[6] += y.z; a[7] += y.w;
      if (EPI == EPI_SILU_MUL) {
        const float4* q = p + 4;  // +16 floats: the matching up columns
        float4 z = q[0], w = q[1];
        b[0] += z.x; b[1] += z.y; b[2] += z.z; b[3] += z.w;
        b[4] += w.x; b[5] += w.y; b[6] += w.z; b[7] += w.w;
      }
    }
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (EPI == EPI_NONE) {
        o[j] = pack2(a[2 * j], a[2 * j + 1]);
      } else {
        const float g0 = bf2f(f2bf(a[2 * j])), g1 = bf2f(f2bf(a[2 * j + 1]));
        const float s0 = bf2f(f2bf(g0 / (1.f + __expf(-g0))));
        const float s1 = bf2f(f2bf(g1 / (1.f + __expf(-g1))));
        o[j] = pack2(s0 * bf2f(f2bf(b[2 * j])), s1 * bf2f(f2bf(b[2 * j + 1])));
      }
    }
    *reinterpret_cast<u32x4*>(C + (size_t)r * ldc + j0) = o;
  }
}

template <int BM, int BN, int WM, int WN, int EPI, bool GROUPED>
static void run_cfg(const uint16_t* A, int lda, const uint16_t* B, int ldb, uint16_t* C, int ldc,
                    float* ws, int M, int N, int K, int splits, int k_chunk, const int* offsets,
                    int n_groups, int m_tiles, hipStream_t st) {
  constexpr int T = WM * WN * 64;
  const size_t lds_stage = 2 * (size_t)(BM + BN) * kBK * 2;
  const size_t lds_epi = (size_t)BM * (BN + 4) * 4;
  const size_t lds = lds_stage > lds_epi ? lds_stage : lds_epi;
  auto kern = gemm_kernel<BM, BN, WM, WN, EPI, GROUPED>;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  dim3 grid((N + BN - 1) / BN, m_tiles, splits);
  kern<<<grid, T, lds, st>>>(A, lda, B, ldb, C, ldc, ws, M, N, K, k_chunk, offsets, n_groups);
  if (splits > 1) {
    const int outw = EPI == EPI_NONE ? N : N / 2;
    const long total = (long)M * (outw / 8);
    const int g = (int)std::min<long>((total + 255) / 256, 4096);
    splitk_reduce_kernel<EPI><<<g, 256, 0, st>>>(C, ldc, ws, M, N, splits);
  }
}

// Host-side config choice.  Returns the workspace floats needed (0 if none) when
// ws == nullptr && query, else launches.
template <int EPI, bool GROUPED>
static long dispatch(const uint16_t* A, int lda, const uint16_t* B, int ldb, uint16_t* C, int ldc,
                     float* ws, long ws_floats, int M, int N, int K, const int* offsets,
                     int n_groups, int max_rows_per_group, hipStream_t st, bool query) {
  // pick the tile by the (per-group) row count
  const int mrows = GROUPED ? max_rows_per_group : M;
  int BM, BN;
  if (mrows <= 64) { BM = 64; BN = 64; }
  else if (mrows <= 128) { BM = 128; BN = 64; }
  else if (mrows <= 256 || GROUPED) { BM = 256; BN = 64; }
  else { BM = 256; BN = 128; }
  const int n_tiles = (N + BN - 1) / BN;
  int m_tiles = GROUPED ? (M + BM - 1) / BM + n_groups : (M + BM - 1) / BM;
  int splits = 1, k_chunk = K;
  const long tiles = (long)n_tiles * (GROUPED ? (M + BM - 1) / BM : m_tiles);
  if (!GROUPED && tiles < 160 && K >= 1024) {
    splits = (int)std::min<long>(8, std::max<long>(1, 256 / tiles));
    k_chunk = ((K / splits + kBK - 1) / kBK) * kBK;
    splits = (K + k_chunk - 1) / k_chunk;
  }
  const long need = splits > 1 ? (long)splits * M * N : 0;
  if (query) return need;
  if (need > ws_floats) { splits = 1; k_chunk = K; }  // no workspace: single pass
#define MLOP_GEMM(bm, bn, wm, wn)                                                                   \
  run_cfg<bm, bn, wm, wn, EPI, GROUPED>(A, lda, B, ldb, C, ldc, ws, M, N, K, splits, k_chunk,      \
                                        offsets, n_groups, m_tiles, st)
  if (BM == 64) MLOP_GEMM(64, 64, 1, 4);
  else if (BM == 128) MLOP_GEMM(128, 64, 2, 2);
  else if (BN == 64) MLOP_GEMM(256, 64, 4, 1);
  else MLOP_GEMM(256, 128, 4, 2);
#undef MLOP_GEMM
  return need;
}

long gemm_workspace_floats(int M, int N, int K, int epi) {
  return epi == EPI_NONE
             ? dispatch<EPI_NONE, false>(nullptr, 0, nullptr, 0, nullptr, 0, nullptr, 0, M, N, K,
                                         nullptr, 0, 0, nullptr, true)
             : dispatch<EPI_SILU_MUL, false>(nullptr, 0, nullptr, 0, nullptr, 0, nullptr, 0, M, N,
                                             K, nullptr, 0, 0, nullptr, true);
}

void launch_gemm(const void* A, int lda, const void* B, int ldb, void* C, int ldc, float* ws,
                 long ws_floats, int M, int N, int K, int epi, hipStream_t st) {
  if (M == 0) return;
  if (epi == EPI_NONE)
    dispatch<EPI_NONE, false>((const uint16_t*)A, lda, (const uint16_t*)B, ldb, (uint16_t*)C, ldc,
                              ws, ws_floats, M, N, K, nullptr, 0, 0, st, false);
  else
    dispatch<EPI_SILU_MUL, false>((const uint16_t*)A, lda, (const uint16_t*)B, ldb, (uint16_t*)C,
                                  ldc, ws, ws_floats, M, N, K, nullptr, 0, 0, st, false);
}

void launch_grouped_gemm(const void* A, const void* B, void* C, const int* offsets, int n_groups,
                         int M, int N, int K, int max_rows, int epi, hipStream_t st) {
  if (M == 0) return;
  if (epi == EPI_NONE)
    dispatch<EPI_NONE, true>((const uint16_t*)A, K, (const uint16_t*)B, K, (uint16_t*)C, N,
                             nullptr, 0, M, N, K, offsets, n_groups, max_rows, st, false);
  else
    dispatch<EPI_SILU_MUL, true>((const uint16_t*)A, K, (const uint16_t*)B, K, (uint16_t*)C, N / 2,
                                 nullptr, 0, M, N, K, offsets, n_groups, max_rows, st, false);
}

}  // namespace mlop
