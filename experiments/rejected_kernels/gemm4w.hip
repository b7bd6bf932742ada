// K1 bf16 GEMM, large-M body: 256 x 256 tile, FOUR waves (one per SIMD), 128 x 128 outputs
// per wave (64 accumulators of 16x16, the AGPR half of the 512-entry register file).
//
//   C[M, N] = A[M, K] . B[N, K]^T      (A activations, B weights [out, in])
//
// Why this shape (profiles/r03_gemm_baseline_pmc.md): the two-group ping-pong kernel
// (gemm.hip gemm_pp_kernel, 8 waves x 128 x 64) reads 192 KB of LDS per CU per 64-deep
// K-step and meets 8 barriers per K-step; at 4096^3 it spends 30 % of its wave cycles parked
// and takes 20 % more cycles than hipBLASLt's 4-wave 256x256 kernel.  A 128 x 128 wave tile
// reads 2/3 of the LDS bytes per MFMA (A and B panels of 128 rows each) and needs ONE barrier
// per K-step; with one wave per SIMD the latency has to be hidden inside the wave:
//
//   * K is walked in 32-deep steps (one v_mfma_f32_16x16x32_bf16 per 16x16 block and step:
//     64 MFMAs = 1024 matrix cycles per wave per step);
//   * a FIVE-slot LDS-DMA ring (5 x 32 KB = 160 KB, the whole LDS): step s+4 is issued while
//     step s computes, so every step's bytes have ~3 steps (~3000 cycles) to land; each wave
//     issues 8 x 1 KiB pieces per step, ALWAYS (the last steps re-load the final K-step into
//     free slots), so one constant counted vmcnt(16) retires step s+1 at the top of step s;
//   * fragments are double-buffered in registers: step s+1's 16 ds_read_b128 (and the step's 8
//     DMA pieces) are threaded 1 : 2 between the first 32 of step s's 64 MFMAs
//     (sched_group_barrier), so they have landed long before step s+1's first MFMA;
//   * ONE raw s_barrier per step (stage s+1 visible everywhere; slot s-1 free for step s+4);
//   * LDS image: 16-row x 64-B pieces written lane-linearly by LDS-DMA; 16-B chunk c of row r
//     sits at slot c ^ g(r), g(r) = (4 - ((r >> 2) & 3)) & 3, applied to the SOURCE address
//     (rule 21).  Each 16-lane group of a fragment ds_read_b128 (rows r..r+15, one chunk)
//     then covers all 16 slots of the 256-B bank row: conflict-free;
//   * epilogue: each wave stages its bf16 128 x 128 tile in the (drained) ring and writes
//     16-B coalesced rows; SiLU-mul (gate/up interleaved in groups of 16) and the QKV RoPE +
//     paged-cache epilogue (rope_epi.h) as in gemm.hip.
//   * XCD-aware tile order (T1, bijective) with bands of group_m m-tiles sharing a B panel.
#include "common.h"
#include "launch.h"
#include "rope_epi.h"

namespace mlop {

namespace w4 {
constexpr int BM = 256, BN = 256, BK = 32, NST = 5, NT = 256;
constexpr int STAGE = (BM + BN) * BK;  // bf16 elements per ring slot (32 KB)
constexpr size_t LDS_BYTES = (size_t)NST * STAGE * 2;  // 160 KB
static_assert(LDS_BYTES <= 163840, "LDS budget");
__device__ __forceinline__ int g4(int r) { return (4 - ((r >> 2) & 3)) & 3; }
}  // namespace w4

enum { W4_NONE = 0, W4_SILU_MUL = 1, W4_ROPE = 3 };

template <int EPI>
__global__ void __launch_bounds__(256, 1) gemm4w_kernel(const uint16_t* __restrict__ A, int lda,
                                                        const uint16_t* __restrict__ B, int ldb,
                                                        uint16_t* __restrict__ C, int ldc, int M, int N,
                                                        int K, int n_tiles_x, int m_tiles, int group_m,
                                                        RopeEpi re) {
  using namespace w4;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;

  // XCD-aware tile order: each XCD a contiguous range of logical tiles; bands of group_m
  // m-tiles, m fastest inside a band, so a B panel is reused while L2-resident.  Speed only.
  const int G = gridDim.x, L = blockIdx.x;
  const int q = G >> 3, rr = G & 7, xcd = L & 7, xs = L >> 3;
  const int lid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + xs;
  const int band = lid / (group_m * n_tiles_x), in_band = lid % (group_m * n_tiles_x);
  const int gm_here = min(group_m, m_tiles - band * group_m);
  const int m0 = (band * group_m + in_band % gm_here) * BM;
  int n0 = (in_band / gm_here) * BN;
  if constexpr (EPI == W4_ROPE) n0 = (n_tiles_x - 1) * BN - n0;  // slow V-head tiles first
  const int nk = K / BK;

#ifdef W4_GLDS
  // (LDS-DMA staging: measured slower, every piece stalls the lone wave ~100 cycles)
#error "W4_GLDS variant removed"
#endif
  // Register staging: wave w loads A rows w*64 .. w*64+63 and the same B rows of each 32-deep
  // step (4 + 4 global_load_dwordx4, lane -> row lane>>2 of a 16-row piece, 16-B chunk lane&3,
  // coalesced 64-B row segments) into one of two register sets, and writes them to the LDS
  // slot at chunk position (chunk ^ g(row)) with ds_write_b128 two steps later.
  const int prow = lane >> 2, pch = lane & 3;
  const int rowA = m0 + wid * 64 + prow, rowB = n0 + wid * 64 + prow;
  const uint16_t* gA[4];
  const uint16_t* gB[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    gA[i] = A + (size_t)min(rowA + 16 * i, M - 1) * lda + pch * 8;
    gB[i] = B + (size_t)min(rowB + 16 * i, N - 1) * ldb + pch * 8;
  }
  const int woff = (wid * 64 + prow) * BK + ((pch ^ g4(prow)) << 3);  // + i * 16 rows
  auto gload = [&](bf16x8 (&g)[8], int ks) {
#pragma unroll
    for (int i = 0; i < 4; ++i) g[i] = *reinterpret_cast<const bf16x8*>(gA[i] + ks * BK);
#pragma unroll
    for (int i = 0; i < 4; ++i) g[4 + i] = *reinterpret_cast<const bf16x8*>(gB[i] + ks * BK);
  };
  auto swrite = [&](int slot, const bf16x8 (&g)[8]) {
    uint16_t* base = smem + slot * STAGE + woff;
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<bf16x8*>(base + i * 16 * BK) = g[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<bf16x8*>(base + BM * BK + i * 16 * BK) = g[4 + i];
  };
  // fragment read offsets (elements): lane -> row lane&15 of a 16-row block, chunk lane>>4
  const int r16 = lane & 15;
  const int foff = r16 * BK + (((lane >> 4) ^ g4(r16)) << 3);
  const int offA = wm * 128 * BK + foff, offB = BM * BK + wn * 128 * BK + foff;
  auto rdA = [&](int slot, int i) {
    return *reinterpret_cast<const bf16x8*>(smem + slot * STAGE + offA + i * 16 * BK);
  };
  auto rdB = [&](int slot, int j) {
    return *reinterpret_cast<const bf16x8*>(smem + slot * STAGE + offB + j * 16 * BK);
  };

  // no zero-initialised accumulators: step 0's MFMAs take a zero C operand, so every
  // loop-carried accumulator is an MFMA result (hipcc otherwise carried part of the
  // 256 accumulators in VGPRs and shuffled them through AGPRs every iteration)
  f32x4 acc[8][8];

  // prologue: steps 0, 1 to LDS slots 0, 1; steps 2, 3 in the two register sets
  bf16x8 g0[8], g1[8];
  gload(g0, 0);
  gload(g1, min(1, nk - 1));
  swrite(0, g0);
  gload(g0, min(2, nk - 1));
  swrite(1, g1);
  gload(g1, min(3, nk - 1));
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();
  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) fa0[i] = rdA(0, i);
#pragma unroll
  for (int j = 0; j < 8; ++j) fb0[j] = rdB(0, j);

  // one step: step s+1's fragments from LDS, step s+2's staged registers into the free slot,
  // step s+4's global loads into those registers, the 64 MFMAs of step s threaded between;
  // ONE barrier (behind lgkmcnt(0): this wave's slot writes are done) ends the step
  auto step = [&](int s, bf16x8 (&fa)[8], bf16x8 (&fb)[8], bf16x8 (&ga)[8], bf16x8 (&gb)[8],
                  bf16x8 (&g)[8], bool first) {
    const int nslot = (s + 1) % 3;
#pragma unroll
    for (int j = 0; j < 8; ++j) gb[j] = rdB(nslot, j);
#pragma unroll
    for (int i = 0; i < 8; ++i) ga[i] = rdA(nslot, i);
    swrite((s + 2) % 3, g);  // hipcc waits for these loads (issued two steps ago) first
    gload(g, min(s + 4, nk - 1));
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = mfma16(fa[i], fb[j], first ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[i][j]);
#ifndef W4_NO_SGB
    // 8 x [2 MFMA, DS read, 2 MFMA, DS read | DS write, VMEM] then the last 32 MFMAs
#pragma unroll
    for (int gi = 0; gi < 8; ++gi) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // DS write
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 32, 0);
#endif
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
  };
  step(0, fa0, fb0, fa1, fb1, g0, true);
  step(1, fa1, fb1, fa0, fb0, g1, false);
  for (int s = 2; s < nk; s += 2) {
    step(s, fa0, fb0, fa1, fb1, g0, false);
    step(s + 1, fa1, fb1, fa0, fb0, g1, false);
  }
  __syncthreads();  // ring read everywhere: it becomes the C staging area (the tail loads
                    // of clamped steps land in registers only)

  const int rows_here = min(BM, M - m0);
  if constexpr (EPI == W4_ROPE) {
    // the whole 256 x 256 bf16 tile (two heads), then rotate / scatter per head
    constexpr int LDR = BN + 8;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * 128 + i * 16 + 4 * (lane >> 4) + r;
#pragma unroll
        for (int j = 0; j < 8; ++j) smem[row * LDR + wn * 128 + j * 16 + r16] = f2bf(acc[i][j][r]);
      }
    __syncthreads();
    auto at = [&](int r, int c) { return bf2f(smem[r * LDR + c]); };
    rope_tile_store<NT>(at, n0 / 128, 2, m0, rows_here, re, tid);
    return;
  }
  constexpr int OW = EPI == W4_NONE ? 128 : 64;  // this wave's output columns
  constexpr int LD = OW + 8;
  uint16_t* sC = smem + wid * 128 * LD;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = i * 16 + 4 * (lane >> 4) + r;
      if constexpr (EPI == W4_NONE) {
#pragma unroll
        for (int j = 0; j < 8; ++j) sC[row * LD + j * 16 + r16] = f2bf(acc[i][j][r]);
      } else {
#pragma unroll
        for (int jp = 0; jp < 4; ++jp) {
          const float g = acc[i][2 * jp][r], u = acc[i][2 * jp + 1][r];
          sC[row * LD + jp * 16 + r16] = f2bf(silu_bf(g) * bf2f(f2bf(u)));
        }
      }
    }
  __syncthreads();
  constexpr int CPR = OW / 8;  // 16-B chunks per row
  const int out_c0 = EPI == W4_NONE ? n0 + wn * 128 : (n0 + wn * 128) / 2;
  const int out_n = EPI == W4_NONE ? N : N / 2;
#pragma unroll 4
  for (int c = lane; c < 128 * CPR; c += 64) {
    const int row = c / CPR, cc = (c % CPR) * 8;
    const int gm = m0 + wm * 128 + row, gn = out_c0 + cc;
    if (gm < M && gn < out_n)
      *reinterpret_cast<u32x4*>(C + (size_t)gm * ldc + gn) = *reinterpret_cast<const u32x4*>(sC + row * LD + cc);
  }
}

template <int EPI>
static void run_w4(const uint16_t* A, int lda, const uint16_t* B, int ldb, uint16_t* C, int ldc, int M, int N,
                   int K, int group_m, hipStream_t st, const RopeEpi& re) {
  auto kern = gemm4w_kernel<EPI>;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)w4::LDS_BYTES);
    attr = true;
  }
  const int gx = N / 256, gy = (M + 255) / 256;
  const int gm = std::max(1, std::min(group_m, gy));
  kern<<<gx * gy, 256, w4::LDS_BYTES, st>>>(A, lda, B, ldb, C, ldc, M, N, K, gx, gy, gm, re);
}

// Shapes the four-wave body takes: N a multiple of 256, K of 64 (two 32-deep steps per
// unrolled iteration), row strides 16-B aligned.
bool gemm4w_supported(int M, int N, int K, int lda, int ldb) {
  return M > 0 && N % 256 == 0 && K % 64 == 0 && K >= 128 && lda % 8 == 0 && ldb % 8 == 0;
}

static int g_w4_group_m = [] {
  const char* e = getenv("MLOP_GEMM_W4_GROUP_M");
  return e ? atoi(e) : 4;
}();

bool launch_gemm4w(const void* A, int lda, const void* B, int ldb, void* C, int ldc, int M, int N, int K,
                   int epi, hipStream_t st, const RopeEpi* re) {
  if (!gemm4w_supported(M, N, K, lda, ldb)) return false;
  const auto* a = static_cast<const uint16_t*>(A);
  const auto* b = static_cast<const uint16_t*>(B);
  auto* c = static_cast<uint16_t*>(C);
  switch (epi) {
    case W4_NONE: run_w4<W4_NONE>(a, lda, b, ldb, c, ldc, M, N, K, g_w4_group_m, st, RopeEpi{}); return true;
    case W4_SILU_MUL: run_w4<W4_SILU_MUL>(a, lda, b, ldb, c, ldc, M, N, K, g_w4_group_m, st, RopeEpi{}); return true;
    case W4_ROPE:
      if (!re || N % 256) return false;
      run_w4<W4_ROPE>(a, lda, b, ldb, nullptr, 0, M, N, K, g_w4_group_m, st, *re);
      return true;
    default: return false;
  }
}

}  // namespace mlop
