// bf16 GEMM on MFMA for gfx950 (K1 prefill / K2 decode / K13 MoE grouped).
//
//   C[M, N] = A[M, K] . B[N, K]^T        (A: activations row-major, B: weights [out, in])
//
// Structure (cdna_hip_programming.md §5 "glds vs register staging", "Pipelining
// across barriers"):
//   * a workgroup owns a BM x BN tile; K is walked in BK = 64 steps;
//   * BOTH operands stream global -> LDS with global_load_lds_dwordx4 (LDS-DMA,
//     no VGPR staging) into a 3-deep ring: two k-steps stay in flight while the
//     MFMAs consume the third;
//   * one raw s_barrier per k-step, preceded by a COUNTED vmcnt (never 0 in the
//     steady state) — __syncthreads() would drain the DMA queue (its fence emits
//     vmcnt(0));
//   * the LDS image is lane-linear per 1 KiB piece (8 rows x 128 B), XOR-swizzled
//     through the SOURCE address: 16-B chunk c of row r sits at slot c ^ ((r>>1)&7),
//     so the 16 rows a ds_read_b128 lane group reads hit 16 different bank slots
//     (T2, rule 21: swizzle the source and the read, never the LDS destination);
//   * all LDS lives in ONE extern __shared__ array (a second object can make hipcc
//     emit vmcnt(0) before every ds_read: §5 item 4(a));
//   * waves WM x WN, each owning (BM/WM) x (BN/WN) as 16x16 accumulators fed by
//     v_mfma_f32_16x16x32_bf16.
//
// Decode (M <= 256) is weight-streaming: BM covers the batch so each weight byte
// is fetched from HBM once; when the N tiles cannot fill 256 CUs, K is split over
// blockIdx.z and fp32 slabs are combined by a reduce kernel that also applies
// the epilogue — optionally fused with the decoder's residual add + RMSNorm
// (launch-boundary reduce, §5 "Projection GEMM at M = 256" item 2).
//
// Epilogues (fp32 LDS copy of the tile, 16-B coalesced stores):
//   EPI_NONE      C = bf16(acc)
//   EPI_SILU_MUL  B rows gate/up interleaved in groups of 16, C[:, j] = silu(g_j) * u_j (N/2 cols)
//   EPI_ROPE      QKV projection: RoPE on q/k heads + q_out / paged K,V cache stores from the
//                 staged tile (RopeEpi, launch.h); needs whole 128-wide heads per staged chunk
// Grouped mode (MoE K13): A rows sorted by expert, offsets[e]..offsets[e+1];
// B = W[e] ([E, N, K]); blockIdx.y enumerates (expert, m-tile) pairs on device.
#include "common.h"
#include "launch.h"
#include "rope_epi.h"

namespace mlop {

enum { EPI_NONE = 0, EPI_SILU_MUL = 1, EPI_ROPE = 3 };
constexpr int kBK = 64;
constexpr int kStages = 3;
constexpr int kMaxSplits = 8;  // plan(): split-K factors are at most 8

// 16-B slot of chunk c in image row r is c ^ swz(r).  Two 128-B rows share one
// 256-B bank row, so (r>>1)&7 (not r&7) makes the 16 rows of a ds_read_b128 lane
// group land on 16 distinct slots: (r&1) picks the half, swz the slot in it.
__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }



// Mid-M norm chain (5-64 rows, launch_mid_res_ss): the O / down projection's split-K GEMM
// finishes itself.  Every split stored its fp32 partial write-through (sc1), waited for it,
// met its workgroup at a barrier, and one lane draws a relaxed agent-scope ticket on the
// tile's counter; the split that draws the last ticket reads the partials with sc1 loads only
// (re.mid_acq 0: MI355X_MICROARCH.md "Valid forms", sc1 stores, every storing wave's vmcnt(0)
// and the workgroup barrier before the ONE lane's ticket, sc1 loads of every handed-off byte),
// or with plain loads behind one agent acquire (re.mid_acq 1: attention.hip's split-KV combine
// protocol, for kernels with several workgroups per CU), and
//   * sums the tile's slabs in split order (splitk_add_rmsnorm's order and rounding: the
//     residual comes out bit-identical to the unfused path), residual = bf16(res + bf16(y));
//   * stores each row's sum of squares over the tile's BN columns (sc1) to the partials
//     [M][gx] past the slabs, then draws the row band's ticket;
// the band's last tile sums every row's partials in tile order into ss_tot[M], which the
// consumers (gate_up / QKV) turn into their rows' RMSNorm factors.  Counters: [gx * gy) tiles,
// then gy bands, re-armed by their last arriver.
// buffer loads with a fixed cache policy (AUX 16: sc1)
template <int AUX>
__device__ __forceinline__ u32x4 ld_b128(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, AUX));
}
template <int AUX>
__device__ __forceinline__ float ld_f32(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, AUX));
}

template <int BM, int BN, int T>
__device__ __forceinline__ void mid_chain_finish(uint16_t* __restrict__ C, int ldc, float* __restrict__ ws, int M,
                                                 int N, int m0, int n0, int rows_here, int bx, int by, int gx, int gy,
                                                 int n_splits, const RopeEpi& re, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every wave's partial stored (and its LDS ring reads retired: flag reuses it)
  const int tid = threadIdx.x;
  int* tcnt = re.ss_cnt + by * gx + bx;
  if (tid == 0) flag[0] = __hip_atomic_fetch_add(tcnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n_splits - 1;
  __syncthreads();
  if (!flag[0]) return;
  const bool acq = re.mid_acq != 0;
  if (tid == 0) {
    if (acq) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __hip_atomic_store(tcnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (acq) __syncthreads();
  constexpr int VPR = BN / 8;  // 8-column vectors per tile row
  constexpr int RPP = T / VPR;  // rows per pass
  static_assert(T % VPR == 0 && VPR <= 64 && (VPR & (VPR - 1)) == 0, "row lanes");
  float* ssp = ws + (size_t)n_splits * M * N;  // [M][gx] row partials
  const auto rsS = __builtin_amdgcn_make_buffer_rsrc(ssp, 0, 0x7fffffff, 0x00020000);
  const auto rsW = __builtin_amdgcn_make_buffer_rsrc(ws, 0, 0x7fffffff, 0x00020000);
  for (int r0 = 0; r0 < BM; r0 += RPP) {
    const int r = r0 + tid / VPR, c = (tid % VPR) * 8;
    const int m = m0 + r, n = n0 + c;
    const bool ok = r < rows_here && n < N;
    float ssq = 0.f;
    if (ok) {
      // every slab's two loads in flight together (a runtime-bound loop waits out one memory
      // round trip per split), then summed in split order
      u32x4 x[kMaxSplits], y[kMaxSplits];
#pragma unroll
      for (int sp = 0; sp < kMaxSplits; ++sp)
        if (sp < n_splits) {
          const uint32_t off = (uint32_t)((((size_t)sp * M + m) * N + n) * 4);
          x[sp] = acq ? ld_b128<0>(rsW, off) : ld_b128<16>(rsW, off);
          y[sp] = acq ? ld_b128<0>(rsW, off + 16u) : ld_b128<16>(rsW, off + 16u);
        }
      float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sp = 0; sp < kMaxSplits; ++sp)
        if (sp < n_splits) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            a[e] += __uint_as_float(x[sp][e]);
            a[4 + e] += __uint_as_float(y[sp][e]);
          }
        }
      uint16_t* rp = C + (size_t)m * ldc + n;
      const u32x4 res = *reinterpret_cast<const u32x4*>(rp);
      u32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o[j] = pack2(bf2f(f2bf(a[2 * j])) + lo_bf(res[j]), bf2f(f2bf(a[2 * j + 1])) + hi_bf(res[j]));
        const float h0 = lo_bf(o[j]), h1 = hi_bf(o[j]);
        ssq += h0 * h0 + h1 * h1;
      }
      *reinterpret_cast<u32x4*>(rp) = o;
    }
#pragma unroll
    for (int o2 = VPR / 2; o2 > 0; o2 >>= 1) ssq += __shfl_xor(ssq, o2);
    if (ok && (tid % VPR) == 0)
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(ssq), rsS, (uint32_t)(((size_t)m * gx + bx) * 4), 0,
                                            16 /* sc1 */);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* bcnt = re.ss_cnt + gx * gy + by;
  if (tid == 0) flag[1] = __hip_atomic_fetch_add(bcnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gx - 1;
  __syncthreads();
  if (!flag[1]) return;
  if (tid == 0) {
    if (acq) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __hip_atomic_store(bcnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (acq) __syncthreads();
  // row totals: L = T / BM lanes per row, each summing the partials b = l, l + L, ... (loads
  // batched 8 at a time), then a fixed shuffle tree over the L lanes: deterministic, and no
  // chain of gx dependent memory round trips
  constexpr int L = T / BM >= 64 ? 64 : T / BM;
  static_assert(L >= 1 && (L & (L - 1)) == 0, "lanes per row");
  for (int r0 = 0; r0 < BM; r0 += T / L) {
    const int r = r0 + tid / L, l = tid % L;
    float sum = 0.f;
    if (r < rows_here) {
      const uint32_t row_off = (uint32_t)((size_t)(m0 + r) * gx * 4);
      for (int b0 = l; b0 < gx; b0 += 8 * L) {
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int b = b0 + k * L;
          v[k] = b >= gx ? 0.f : acq ? ld_f32<0>(rsS, row_off + (uint32_t)b * 4u) : ld_f32<16>(rsS, row_off + (uint32_t)b * 4u);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) sum += v[k];
      }
    }
#pragma unroll
    for (int o2 = L / 2; o2 > 0; o2 >>= 1) sum += __shfl_xor(sum, o2);
    if (r < rows_here && l == 0) re.ss_tot[m0 + r] = sum;
  }
}

template <int BM, int BN, int WM, int WN, int EPI, bool GROUPED, int STAGES = 3, bool SETPRIO = false>
__global__ void __launch_bounds__(WM * WN * 64) gemm_kernel(
    const uint16_t* __restrict__ A, int lda, const uint16_t* __restrict__ B, int ldb,
    uint16_t* __restrict__ C, int ldc, float* __restrict__ ws, int M, int N, int K, int k_chunk,
    const int* __restrict__ offsets, int n_groups, int n_tiles_x, int m_tiles_y, int n_splits,
    RopeEpi re) {
  constexpr int NW = WM * WN, T = NW * 64;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int NP = (BM + BN) / 8;  // 1-KiB pieces (8 rows x 128 B) per stage
  static_assert(NP % NW == 0, "pieces must divide the waves");
  constexpr int PPW = NP / NW;        // LDS-DMA instructions per wave per stage
  constexpr int STAGE = (BM + BN) * kBK;  // bf16 elements per stage
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  // XCD-aware remap (T1, bijective form): the 1-D grid is dealt round-robin over
  // the 8 XCDs, so give each XCD a CONTIGUOUS range of logical tiles ordered
  // (split, m-tile, n-tile): tiles sharing an A panel / K-chunk share an L2.
  // Speed only — correctness never depends on placement.
  const int G = gridDim.x, L = blockIdx.x;
  const int q = G >> 3, rr = G & 7, xcd = L & 7, slot = L >> 3;
  const int lid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + slot;
  const int gx = n_tiles_x;
  // grouped: the (expert, m-tile) slot is the FAST index, so the slots left empty by a
  // routing (the grid is sized for the worst case, m_tiles + n_groups) are spread over
  // every XCD's contiguous range instead of idling the XCDs that drew the tail slots
  const int bx = GROUPED ? (lid / m_tiles_y) % gx : lid % gx;
  const int by = GROUPED ? lid % m_tiles_y : (lid / gx) % m_tiles_y;
  const int bz = lid / (gx * m_tiles_y);
  const int n0 = bx * BN;
  int m0 = by * BM, m_end = M;
  const uint16_t* Bg = B;
  if constexpr (GROUPED) {
    int t = by, e = 0;
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
  const int kbeg = bz * k_chunk;
  const int kend = min(K, kbeg + k_chunk);
  const int nk = (kend - kbeg) / kBK;
  const bool split = n_splits > 1;

  // per-lane source row / chunk of each piece this wave issues (k advances by kBK)
  const int prow = lane >> 3;                  // row inside the 8-row piece
  const uint16_t* src[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int p = wid + i * NW;
    const int r = p * 8 + prow;
    const int pchunk = (lane & 7) ^ swz(r);     // source chunk for LDS slot (lane & 7)
    if (r < BM) {
      int gr = min(m0 + r, m_end - 1);
      if (GROUPED && re.a_rows != nullptr) gr = re.a_rows[gr];
      src[i] = A + (size_t)gr * lda + kbeg + pchunk * 8;
    } else {
      const int gn = min(n0 + r - BM, N - 1);
      src[i] = Bg + (size_t)gn * ldb + kbeg + pchunk * 8;
    }
  }
  // weight pieces non-temporal when re.b_nt (wave-uniform: a piece is A or B by its index)
  const bool b_nt = re.b_nt != 0;
  auto issue = [&](int buf, int kt) {
    uint16_t* base = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int p = wid + i * NW;
      if (b_nt && p >= BM / 8)
        __builtin_amdgcn_global_load_lds((const void*)(src[i] + kt * kBK),
                                         (lds_void_t*)(base + p * 512), 16, 0, 2 /* nt */);
      else
        __builtin_amdgcn_global_load_lds((const void*)(src[i] + kt * kBK),
                                         (lds_void_t*)(base + p * 512), 16, 0, 0);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) issue(s, s);
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt must have landed; the STAGES-2 younger stages may stay in flight
    // the STAGES-2 younger stages may stay in flight (fewer near the end: drain)
    if (STAGES >= 3 && kt + STAGES - 2 < nk) wait_vmcnt<(STAGES >= 3 ? (STAGES - 2) * PPW : 0)>();
    else wait_vmcnt<0>();
    raw_barrier();  // stage kt visible to all waves; stage kt-1's buffer free
    if (kt + STAGES - 1 < nk) issue((kt + STAGES - 1) % STAGES, kt + STAGES - 1);
    const uint16_t* sA = smem + (kt % STAGES) * STAGE;
    const uint16_t* sB = sA + BM * kBK;
    if constexpr (SETPRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk * 4 + (lane >> 4);
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * WTM + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(sA + r * kBK + ((ch ^ swz(r)) << 3));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * WTN + j * 16 + (lane & 15);
        bfr[j] = *reinterpret_cast<const bf16x8*>(sB + r * kBK + ((ch ^ swz(r)) << 3));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
    if constexpr (SETPRIO) __builtin_amdgcn_s_setprio(0);
  }

  const int rows_here = min(BM, m_end - m0);
  if (split) {
    // split-K: fp32 partial slab [kz][M][N] (plain stores; reduce kernel in the next launch).
    // Mid norm chain (re.ss_cnt set, launch_mid_res_ss): write-through (sc1) stores, then the
    // last split of the tile finishes it in this launch (mid_chain_finish).
    float* P = ws + (size_t)bz * M * N;
    const bool fix = !GROUPED && re.ss_cnt != nullptr;
    const auto rsP = __builtin_amdgcn_make_buffer_rsrc(P, 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * WTN + j * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ml = wm * WTM + i * 16 + 4 * (lane >> 4) + r;
          if (ml < rows_here && n < N) {
            if (fix)
              __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[i][j][r]), rsP,
                                                    (uint32_t)(((size_t)(m0 + ml) * N + n) * 4), 0, 16 /* sc1 */);
            else if (re.ws_nt & 1) __builtin_nontemporal_store(acc[i][j][r], P + (size_t)(m0 + ml) * N + n);
            else P[(size_t)(m0 + ml) * N + n] = acc[i][j][r];
          }
        }
      }
    if constexpr (!GROUPED) {
      if (fix) mid_chain_finish<BM, BN, T>(C, ldc, ws, M, N, m0, n0, rows_here, bx, by, gx, m_tiles_y, n_splits, re,
                                           reinterpret_cast<int*>(smem));
    }
    return;
  }
  raw_barrier();  // every wave is done reading the ring before it becomes the C tile
  // the C tile goes through LDS in column chunks of <= 128 (fp32 [BM][EW + 4])
  float* sC = reinterpret_cast<float*>(smem);
  constexpr int EW = BN < 128 ? BN : 128;
  constexpr int LDC = EW + 4;
#pragma unroll
  for (int c0 = 0; c0 < BN; c0 += EW) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = wn * WTN + j * 16 + (lane & 15) - c0;
        if (n >= 0 && n < EW) {
#pragma unroll
          for (int r = 0; r < 4; ++r) sC[(wm * WTM + i * 16 + 4 * (lane >> 4) + r) * LDC + n] = acc[i][j][r];
        }
      }
    __syncthreads();
    if constexpr (EPI == EPI_ROPE) {
      static_assert(EW == 128, "EPI_ROPE stages one whole head per chunk");
      static_assert(BM == 256, "EPI_ROPE tiles are 256 rows");
      auto at = [&](int r, int c) { return bf2f(f2bf(sC[r * LDC + c])); };
      rope_tile_store<T>(at, (n0 + c0) / 128, 1, m0, rows_here, re, tid);
    } else if constexpr (EPI == EPI_NONE) {
      constexpr int VPR = EW / 8;
      for (int v = tid; v < BM * VPR; v += T) {
        const int r = v / VPR, c = (v % VPR) * 8;
        if (r >= rows_here || n0 + c0 + c >= N) continue;
        const float* s = sC + r * LDC + c;
        u32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = pack2(s[2 * j], s[2 * j + 1]);
        *reinterpret_cast<u32x4*>(C + (size_t)(m0 + r) * ldc + n0 + c0 + c) = o;
      }
    } else {
      constexpr int OUTW = EW / 2, VPR = OUTW / 8;
      for (int v = tid; v < BM * VPR; v += T) {
        const int r = v / VPR, j0 = (v % VPR) * 8;
        const int gcol = (j0 / 16) * 32 + (j0 % 16);
        if (r >= rows_here || n0 + c0 + gcol >= N) continue;
        const float* g = sC + r * LDC + gcol;
        const float* u = g + 16;
        // mid norm chain (re.ss_in: the producer's row totals): the row's RMSNorm factor scales
        // the accumulators first (W4_RS's order)
        const float f = re.ss_in != nullptr ? rsqrtf(re.ss_in[m0 + r] * re.ss_inv_k + re.ss_eps) : 1.f;
        u32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          o[j] = pack2(silu_bf(g[2 * j] * f) * bf2f(f2bf(u[2 * j] * f)),
                       silu_bf(g[2 * j + 1] * f) * bf2f(f2bf(u[2 * j + 1] * f)));
        *reinterpret_cast<u32x4*>(C + (size_t)(m0 + r) * ldc + (n0 + c0) / 2 + j0) = o;
      }
    }
    if (c0 + EW < BN) __syncthreads();
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
      if (EPI == EPI_NONE)
        o[j] = pack2(a[2 * j], a[2 * j + 1]);
      else
        o[j] = pack2(silu_bf(a[2 * j]) * bf2f(f2bf(b[2 * j])),
                     silu_bf(a[2 * j + 1]) * bf2f(f2bf(b[2 * j + 1])));
    }
    *reinterpret_cast<u32x4*>(C + (size_t)r * ldc + j0) = o;
  }
}

// split-K reduce fused with the decoder's residual add + RMSNorm (one row per block):
//   y = bf16(sum_s slab[s][r]);  residual[r] = bf16(residual[r] + y);  out[r] = rmsnorm(residual[r]) * w
template <int VPT>
__global__ void __launch_bounds__(512) splitk_add_rmsnorm_kernel(
    uint16_t* __restrict__ out, uint16_t* __restrict__ residual, const float* __restrict__ ws,
    const uint16_t* __restrict__ w, float eps, int M, int N, int splits) {
  __shared__ float scratch[16];
  const int r = blockIdx.x;
  const int nvec = N >> 3;
  float v[VPT][8];
  float ss = 0.f;
  // the norm weights load with the slabs (one memory latency on the chain, not two)
  u32x4 wpre[VPT];
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int vi = threadIdx.x + i * blockDim.x;
    if (vi < nvec) wpre[i] = *reinterpret_cast<const u32x4*>(w + vi * 8);
  }
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int vi = threadIdx.x + i * blockDim.x;
    if (vi < nvec) {
      // every slab's two loads (and the residual's) in flight together: a runtime-bound loop
      // waited out one L2 round trip per split (~5 us per call at batch 8-64, twice per layer)
      float4 x[kMaxSplits], y[kMaxSplits];
#pragma unroll
      for (int s = 0; s < kMaxSplits; ++s)
        if (s < splits) {
          const float4* p = reinterpret_cast<const float4*>(ws + ((size_t)s * M + r) * N + vi * 8);
          x[s] = p[0];
          y[s] = p[1];
        }
      const u32x4 res = *reinterpret_cast<const u32x4*>(residual + (size_t)r * N + vi * 8);
      float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int s = 0; s < kMaxSplits; ++s)
        if (s < splits) {
          a[0] += x[s].x; a[1] += x[s].y; a[2] += x[s].z; a[3] += x[s].w;
          a[4] += y[s].x; a[5] += y[s].y; a[6] += y[s].z; a[7] += y[s].w;
        }
      u32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float s0 = bf2f(f2bf(a[2 * j])) + lo_bf(res[j]);
        const float s1 = bf2f(f2bf(a[2 * j + 1])) + hi_bf(res[j]);
        o[j] = pack2(s0, s1);
        v[i][2 * j] = lo_bf(o[j]);
        v[i][2 * j + 1] = hi_bf(o[j]);
      }
      *reinterpret_cast<u32x4*>(residual + (size_t)r * N + vi * 8) = o;
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  ss = block_sum(ss, scratch);
  const float inv = rsqrtf(ss / (float)N + eps);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int vi = threadIdx.x + i * blockDim.x;
    if (vi < nvec) {
      const u32x4 wv = wpre[i];
      u32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        o[j] = pack2(bf2f(f2bf(v[i][2 * j] * inv)) * lo_bf(wv[j]),
                     bf2f(f2bf(v[i][2 * j + 1] * inv)) * hi_bf(wv[j]));
      *reinterpret_cast<u32x4*>(out + (size_t)r * N + vi * 8) = o;
    }
  }
}

template <int BM, int BN, int STAGES>
constexpr size_t lds_bytes() {
  constexpr size_t ring = (size_t)STAGES * (BM + BN) * kBK * 2;
  constexpr int EW = BN < 128 ? BN : 128;
  constexpr size_t epi = (size_t)BM * (EW + 4) * 4;
  return ring > epi ? ring : epi;
}

// non-temporal weight stream of the decode-shaped GEMMs (gemm_small_nt op; MI355X_MICROARCH.md
// "nt-weights": serving streams 16 GB of other weights between two reads of one matrix, so the
// default policy's L2 / MALL fills are pure cost).  Interleaved on one box: Llama batch 16 +4.4 %,
// batch 64 +2.6 %, Mixtral batch 64 +6.3 % (gate_up at M = 16 / 64 46.1 -> 41.3 / 52.1 -> 47.7 us);
// bit 0 dense one-m-tile launches, bit 1 grouped small tiles, bit 2 grouped ping-pong
static int g_small_nt_flags = 7;
int gemm_small_nt(int set) {
  if (set >= 0) g_small_nt_flags = set;
  return g_small_nt_flags;
}

// non-temporal stores of GEMM outputs the next launch reads (gemm_slab_nt op; not left dirty in
// L2 for the kernel boundary's write-back, MI355X_MICROARCH.md "boundary"): bit 0 the split-K
// slabs (batch 256 +0.6 %, batch 64 neutral), bit 1 the four-wave kernel's C (headline +1.2 %),
// bit 2 the ping-pong kernel's C (Mixtral batch 256 / 1024 and Llama batch 512 +0.3-0.4 %),
// bit 3 the four-wave RoPE epilogue's q / K / V (with attn_kv_nt 3: headline +0.5 % over 5 pairs)
static int g_slab_nt = 15;
static int g_split_target = 512;  // gemm_split_target op: workgroups the split-K of the 16-row tiles aims at
int gemm_split_target(int set) {
  if (set >= 1) g_split_target = set;
  return g_split_target;
}
int gemm_slab_nt(int set) {
  if (set >= 0) g_slab_nt = set;
  return g_slab_nt;
}

template <int BM, int BN, int WM, int WN, int EPI, bool GROUPED, int STAGES, bool SETPRIO>
static void run_cfg(const uint16_t* A, int lda, const uint16_t* B, int ldb, uint16_t* C, int ldc,
                    float* ws, int M, int N, int K, int splits, int k_chunk, const int* offsets,
                    int n_groups, int m_tiles, hipStream_t st, const RopeEpi& re) {
  constexpr int T = WM * WN * 64;
  constexpr size_t lds = lds_bytes<BM, BN, STAGES>();
  static_assert(lds <= 163840, "LDS budget");
  auto kern = gemm_kernel<BM, BN, WM, WN, EPI, GROUPED, STAGES, SETPRIO>;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int gx = (N + BN - 1) / BN;
  const int blocks = gx * m_tiles * splits;
  // non-temporal weights where each weight byte is streamed by ONE workgroup: one m-tile
  // (dense), or the grouped decode tiles (an expert's few routed rows)
  RopeEpi r = re;
  r.b_nt = GROUPED ? (g_small_nt_flags & 2) != 0 && BM <= 64 : (g_small_nt_flags & 1) != 0 && m_tiles == 1;
  r.ws_nt = g_slab_nt;
  kern<<<blocks, T, lds, st>>>(A, lda, B, ldb, C, ldc, ws, M, N, K, k_chunk, offsets, n_groups, gx,
                               m_tiles, splits, r);
}

static int g_small_stages = 3;
int gemm_small_stages(int set) {
  if (set >= 0) g_small_stages = set;
  return g_small_stages;
}

// Row-fitted narrow tiles for M <= 64 (plan()): 0 = the 64 x 64 tile; 32 / 64 = BN with BM the
// batch rounded up to 16 / 32 / 64; 1 (default) = BM fitted, BN and ring depth per shape (no padding rows streamed through the A ring: the 16-row
// tile's 4-stage ring is 10 KB instead of 16, so more workgroups stay resident per CU).
// Default 64: M <= 32 cold projections 6-17 % faster than the 64 x 64 tile (qkv 18.3 -> 15.3 us,
// o+norm 14.9 -> 12.9, gate_up 47.1 -> 45.6, down+norm 32.9 -> 27.3 at M = 16; BN 32 loses:
// profiles/r02_midbatch_decode.md, scripts/run131.sh).  Run-time settable for A/B.
static int g_small_tile = 1;  // 1 = per-shape (plan); 64 x 64 for M 33-64
// ring depth of the grouped (MoE) 64-row tiles on narrow N (the down projection): 6 measured
// neutral on Mixtral batch 32 / 64 (1,651 vs 1,655, 3,142 vs 3,134 tok/s, scripts/run141.sh)
constexpr int g_grouped_small_stages = 3;
int gemm_small_tile(int set) {
  if (set >= 0) g_small_tile = set;
  return g_small_tile;
}

// grouped-plan override (scripts/bench_moe_decode.py compares MoE decode tilings in one process):
// BM, BN, ring stages, K splits; -1 = the planner's own choice.  Only tile shapes launch_plan has
// a grouped config for are accepted.
static int g_gp[4] = {-1, -1, -1, -1};
void gemm_grouped_plan(int bm, int bn, int stages, int splits) {
  if (bm > 0) {
    static const int ok[][2] = {{16, 32}, {16, 64}, {32, 32}, {32, 64}, {64, 32}, {64, 64},
                                {128, 64}, {256, 64}, {256, 128}, {256, 256}};
    bool found = false;
    for (const auto& t : ok) found = found || (t[0] == bm && t[1] == bn);
    if (!found) throw std::runtime_error("gemm_grouped_plan: no grouped config for this tile");
  }
  g_gp[0] = bm, g_gp[1] = bn, g_gp[2] = stages, g_gp[3] = splits;
}

// dense-plan override (scripts/bench_mid_m.py sweeps the mid-M projection tilings in one
// process): variant (0 = gemm_kernel BM x BN, 1 = 256x256 two-stage, 3 = ping-pong, 5 =
// four-wave, 6 = four-wave half height), BM, BN, K splits (plain gemm_kernel only), LDS ring
// depth of the small tiles (0 = the default); -1 = the planner's own choice
static int g_dp[5] = {-1, -1, -1, -1, 0};
void gemm_dense_plan(int variant, int bm, int bn, int splits, int stages) {
  if (variant >= 0 && variant != 0 && variant != 1 && variant != 3 && variant != 5 && variant != 6)
    throw std::runtime_error("gemm_dense_plan: variant must be 0, 1, 3, 5 or 6");
  if (variant == 0) {
    static const int ok[][2] = {{16, 32}, {16, 64}, {32, 32}, {32, 64}, {64, 32}, {64, 64}, {128, 64}, {256, 64}, {256, 128}};
    bool found = false;
    for (const auto& t : ok) found = found || (t[0] == bm && t[1] == bn);
    if (!found) throw std::runtime_error("gemm_dense_plan: no dense config for this tile");
  }
  g_dp[0] = variant, g_dp[1] = bm, g_dp[2] = bn, g_dp[3] = splits, g_dp[4] = stages > 0 ? stages : 0;
}

// large-M kernel choice (plan() variants below), settable at run time (gemm_big_variant op) so
// A/B microbenches run in one process
static int g_big_variant = 5;
int gemm_big_variant(int set) {
  if (set >= 0) g_big_variant = set;
  return g_big_variant;
}
// the grouped <= 32-rows-per-expert rule (plan() below) on / off (gemm_grouped_narrow op)
static int g_grouped_narrow = 1;
int gemm_grouped_narrow(int set) {
  if (set >= 0) g_grouped_narrow = set;
  return g_grouped_narrow;
}
// the planner's half-height four-wave tile (variant 6) on / off (gemm_half_tile op, A/B runs)
static int g_half_tile = 1;
int gemm_half_tile(int set) {
  if (set >= 0) g_half_tile = set;
  return g_half_tile;
}

// ---------------------------------------------------------------------------
// Ping-pong 256x256 GEMM (after cdna_hip_programming.md "The 256^2 8-phase template"):
// 8 waves = 2 wave GROUPS (A halves) x 4 column strips, 128x64 outputs per wave.
// Each K-tile (BK = 64) is 2 phases, one 64x64 half of the wave's outputs x K=64 (32 MFMAs):
//     [ds_read the half's fragments | issue LDS-DMA | drain lgkmcnt]
//     s_barrier; setprio(1) 32 x MFMA setprio(0); s_barrier
// Group 1 executes one extra barrier up front, so it is always one half-phase
// behind group 0: while one group's waves issue LDS reads / DMA, the other
// group's waves (one per SIMD each) keep the matrix cores busy — the barrier
// and LDS latency that idles a single-group loop (27% SQ_WAIT_ANY in
// profiles/r01_gemm_pmc.md) is overlapped by the partner group instead.
// Two LDS buffers (K-tile parity, 2 x 64 KB); the DMA schedule and its vmcnt /
// barrier accounting are in the comment above the K-loop.
//
// GROUPED (MoE K13 at >= 512 rows per expert): the (expert, m-tile) slot is the fast
// tile index (empty slots of the worst-case grid spread over all XCDs), B = W[e] and
// rows stop at offsets[e+1]; everything else is the dense schedule.
// Stream-K tail (plain, non-grouped launches): the T tiles are T / C full rounds on the C
// CUs plus r = T % C tail tiles, and a tail of r < C whole tiles leaves C - r CUs idle for
// a whole tile time (gate_up at M = 2040: 896 tiles = 3.5 rounds, 12.5 % of the kernel).
// The first T - r tiles stay data-parallel (one per workgroup); the r tail tiles' K-tiles
// are dealt as contiguous ranges of `ipw` K-tiles to n_sk more workgroups.  A workgroup
// whose range covers only part of a tile writes its fp32 accumulators to its own slot
// (2 per workgroup: the piece its range starts in, the piece it ends in), releases at
// agent scope and takes a ticket on the tile's counter; the LAST contributor acquires,
// adds the other slots and runs the normal epilogue, then resets the counter for the next
// launch.  Nobody waits on anybody (placement-independent, MI355X_MICROARCH.md
// "Correctness boundaries": dispatch order and co-residency are not assumed).
struct SkArgs {
  int n_dp;     // data-parallel workgroups = tiles before the tail (blockIdx < n_dp)
  int t0;       // first tail tile (logical tile index)
  int ipw;      // K-tiles per stream-K workgroup
  int n_iters;  // r * nk: K-tiles of the whole tail
  float* ws;    // 2 slots x 256 x 256 fp32 per stream-K workgroup
  int* cnt;     // one ticket counter per tail tile, zero between launches
  int n_base;   // first stream-K block (grouped: the worst-case tile count of the grid)
  int cus;      // CUs the split was planned for
  int min_half; // shortest K-range (K-tiles) the planner may cut
  int skip_dead;  // 1: quadrants past the last row issue no MFMAs (MLOP_GEMM_SKIP_DEAD=0: A/B)
  int balance;    // grouped: an expert over c > 1 m-tiles gets c EQUAL row ranges (gemm_grouped_balance)
  int order;      // grouped: 0 = (expert, m-tile) slot fastest, 1 = expert-major (gemm_grouped_order)
};

// d for the r = T % cus tail tiles of a T-tile launch: each is cut into d equal K-ranges
// (d | nk, so no range straddles two tiles), one per extra workgroup, d <= cus / r, when the
// cost model (in K-tile times, calibrated on scripts/bench_proj.py) beats the tail round's nk:
//   nk / d                   the range itself
//   max(2, 0.04 * r * d)     256 KB fp32 partial per workgroup, HBM-bound when all write
//   2 * (d - 1, or d)        the last contributor's slot reads (one CU, ~3 us per slot)
//   1                        a second pipeline fill + ticket
// 0: keep the data-parallel grid.  Host (plain launches) and device (grouped launches, whose
// tile count depends on the routing) evaluate the same function.
__host__ __device__ inline int sk_choose_d(int T, int nk, int cus, int min_half) {
  const int r = T % cus;
  if (r == 0) return 0;
  float best = 0.9f * nk;  // require a 10 % gain on the tail round
  int best_d = 0;
  const int dmax = cus / r < 32 ? cus / r : 32;
  for (int d = 2; d <= dmax; ++d) {
    if (nk % d || nk / d < min_half) continue;
    const float w = 0.04f * r * d;
    const float cost = nk / d + (w > 2.f ? w : 2.f) + 2.f * (d >= 3 ? d : d - 1) + 1.f;
    if (cost < best) {
      best = cost;
      best_d = d;
    }
  }
  return best_d;
}

// Stream-K workgroup Lb (of n_sk starting at block n0) -> its range index, XCD-contiguous:
// blocks are dealt to the 8 XCDs round-robin (block & 7), so consecutive ranges -- which walk
// consecutive tiles and share their A / B panels -- must sit on ONE XCD's L2.  Dealing them
// round-robin made every XCD fetch nearly all of A and B (QKV at M = 2304: 2x slower).
__device__ __forceinline__ int sk_index(int Lb, int n0, int n_sk) {
  const int x = Lb & 7;
  int before = 0;
  for (int y = 0; y < x; ++y) {
    const int first = (y - n0) & 7;  // offset of XCD y's first block in the region
    before += first < n_sk ? (n_sk - first + 7) / 8 : 0;
  }
  return before + (Lb - n0) / 8;
}

template <int EPI, bool GROUPED = false, bool SK = false>
__global__ void __launch_bounds__(512, 1) gemm_pp_kernel(
    const uint16_t* __restrict__ A, int lda, const uint16_t* __restrict__ B, int ldb,
    uint16_t* __restrict__ C, int ldc, int M, int N, int K, int n_tiles_x, int m_tiles, int group_m,
    RopeEpi re, const int* __restrict__ offsets, int n_groups, SkArgs sk) {
  constexpr int BM = 256, BN = 256;
  constexpr int BUF = (BM + BN) * kBK;  // bf16 per K-tile buffer (64 KB)
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2, wc = wid & 3;
  const int Lb = blockIdx.x;
  const int nk = K / kBK;
  // launch geometry: data-parallel tiles [0, n_dp) on blocks [0, n_base), stream-K ranges
  // over the tail tiles [t0, T) on blocks [n_base, n_base + n_sk)
  int n_dp = sk.n_dp, t0 = sk.t0, ipw = sk.ipw, n_iters = sk.n_iters, n_sk = (int)gridDim.x - sk.n_base;
  int S = 0;  // grouped: (expert, m-tile) slots the routing actually filled
  bool expert_major = false;
  if constexpr (GROUPED) {
    int busy = 0;
    for (int e = 0; e < n_groups; ++e) {
      const int c = (offsets[e + 1] - offsets[e] + BM - 1) / BM;
      S += c;
      busy += c > 0;
    }
    // gemm_grouped_order 2 (auto): expert-major from 3 m-tiles per routed expert on average
    // (Mixtral at 765 rows per expert: gate_up -6 %, down -3.5 %; at 256 rows it lost 3.5 %)
    expert_major = sk.order == 1 || (sk.order == 2 && S >= 3 * busy);
    const int T = S * n_tiles_x;
    n_dp = T;
    t0 = T;
    ipw = 1;
    n_iters = 0;
    n_sk = 0;
    if constexpr (SK) {
      const int d = sk_choose_d(T, nk, sk.cus, sk.min_half);
      if (d) {
        const int r = T % sk.cus;
        n_dp = t0 = T - r;
        ipw = nk / d;
        n_iters = r * nk;
        n_sk = r * d;
      }
    }
  }
  const bool dp = !SK || Lb < sk.n_base;
  if (dp ? Lb >= n_dp : Lb - sk.n_base >= n_sk) return;  // whole workgroup, before any barrier

  // tile (logical index) -> origin.  Plain: bands of group_m m-tiles, m fastest within a band
  // (a B panel is reused by group_m consecutive tiles while L2-resident).  Grouped: the
  // routed (expert, m-tile) slot is the fast index, rows stop at offsets[e + 1], B = W[e].
  int m_end = M;
  const uint16_t* Bg = B;
  bool b_once = false;  // grouped: the expert fits one m-tile, its weights are streamed once
  auto tile_origin = [&](int lid, int& m0, int& n0) {
    if constexpr (GROUPED) {
      int e = 0, k = 0, nt = 0;
      if (expert_major) {
        // expert-major (gemm_grouped_order 1): expert e's c_e x n_tiles_x tiles are consecutive
        // lids, its m-tiles fastest, then its n-tiles.  The XCD-contiguous remap then gives each
        // XCD a run of n-tiles of one or two experts: the c_e m-tiles of an n-tile share its B
        // slice, and consecutive n-tiles reuse the same A rows from L2.  (Slot-fastest order put
        // every expert's m-tiles of an n-tile on the XCD at once: each A slice was read once per
        // n-tile from beyond L2.)
        int base = 0;
        for (; e < n_groups; ++e) {
          const int c = (offsets[e + 1] - offsets[e] + BM - 1) / BM;
          if (lid < base + c * n_tiles_x) break;
          base += c * n_tiles_x;
        }
        const int c = (offsets[e + 1] - offsets[e] + BM - 1) / BM;
        k = (lid - base) % c;
        nt = (lid - base) / c;
      } else {
        const int slot = lid % S;
        int before = 0;
        for (; e < n_groups; ++e) {
          const int c = (offsets[e + 1] - offsets[e] + BM - 1) / BM;
          if (slot < before + c) break;
          before += c;
        }
        k = slot - before;
        nt = lid / S;
      }
      const int rows_e = offsets[e + 1] - offsets[e], c = (rows_e + BM - 1) / BM;
      if (sk.balance && c > 1) {
        // c near-equal row ranges instead of c - 1 full tiles + a spill tile: the tiles of one
        // (expert, n-tile) then do near-equal work, stay in step on one XCD (adjacent lids) and
        // share each B K-tile through L2; a 257-row expert was 256 + 1 rows, the spill tile a
        // whole second walk of the B panel at HBM rate (profiles/r06_moe_spill.md).  Inner
        // boundaries sit on 64-row quadrants (the fewest MFMA quadrants, ceil(rows / 64)), each
        // tile at most BM rows.
        auto bnd = [&](int kk) {
          if (kk >= c) return rows_e;
          int b = 64 * (int)(((long)kk * rows_e + 32L * c) / (64L * c));
          b = min(b, BM * kk);
          return max(b, rows_e - BM * (c - kk));
        };
        m0 = offsets[e] + (k > 0 ? bnd(k) : 0);
        m_end = offsets[e] + bnd(k + 1);
      } else {
        m0 = offsets[e] + k * BM;
        m_end = offsets[e + 1];
      }
      n0 = nt * BN;
      Bg = B + (size_t)e * N * ldb;
      b_once = rows_e <= BM;
    } else {
      const int band = lid / (group_m * n_tiles_x), in_band = lid % (group_m * n_tiles_x);
      const int gm_here = min(group_m, m_tiles - band * group_m);
      m0 = (band * group_m + in_band % gm_here) * BM;
      n0 = (in_band / gm_here) * BN;
      // RoPE epilogue: walk each band's n-tiles backwards (the V heads, last columns, first;
      // they were the slow tiles while V pages were dim-major, and the order costs nothing)
      if constexpr (EPI == EPI_ROPE) n0 = (n_tiles_x - 1) * BN - n0;
    }
  };
  // iteration range of this workgroup in K-tiles of the logical tile space
  int it, it_end, m0g = 0, n0g = 0;
  const int s_idx = dp ? 0 : sk_index(Lb, sk.n_base, n_sk);
  if (dp) {
    // XCD-aware remap of the data-parallel part: each XCD a contiguous range of tiles
    const int G = n_dp;
    const int q = G >> 3, rr = G & 7, xcd = Lb & 7, slot = Lb >> 3;
    const int lid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + slot;
    tile_origin(lid, m0g, n0g);
    it = lid * nk;
    it_end = it + nk;
  } else {
    it = t0 * nk + s_idx * ipw;
    it_end = t0 * nk + min((s_idx + 1) * ipw, n_iters);
  }

  f32x4 acc[8][4];
  const int prow = lane >> 3;
  bool first_piece = true;
  do {
    const int tile = SK ? it / nk : 0;
    const int k0 = SK ? it - tile * nk : 0, k1 = SK ? min(nk, k0 + (it_end - it)) : nk;
    it += k1 - k0;
    int m0 = m0g, n0 = n0g;
    if (SK && !dp) tile_origin(tile, m0, n0);
    if (SK && !first_piece) __syncthreads();  // the previous piece's epilogue is done with the LDS
    first_piece = false;
    const int nkp = k1 - k0;

    // DMA sources: half-tile h (0 A rows mi 0 = 0-63 and 128-191, 1 A rows mi 1, 2 B rows
    // 0-127, 3 B rows 128-255) = 16 pieces of 8 rows x 128 B; wave w moves pieces w, w+8.
    // Buffer-form LDS loads (buffer_load_dwordx4 ... lds): the per-lane byte offset into the
    // operand is fixed per tile and the K-tile advance rides in the scalar soffset, so an issue
    // is M0 + one VMEM instruction -- the global form needed a 64-bit VALU address add per
    // issue, serialised through one reused register pair.
    const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, 0x7fffffff, 0x00020000);
    const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)Bg, 0, 0x7fffffff, 0x00020000);
    uint32_t voff[4][2];
#pragma unroll
    for (int h = 0; h < 4; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int r = h < 2 ? i * 128 + h * 64 + wid * 8 + prow : (h & 1) * 128 + (wid + 8 * i) * 8 + prow;
        const int ch = (lane & 7) ^ swz(r);
        // A rows past the tile's last row (the ragged / grouped tail: a spill m-tile of an expert
        // with 256 + a few rows is almost all such rows) load nothing: an offset past the
        // resource's num_records makes the LDS-DMA a dropped out-of-range access, still counted
        // by vmcnt (the counted waits stay exact) but fetching no line.  Their LDS rows hold
        // don't-care values that only ever reach accumulator rows that are never stored.
        const int arow = (GROUPED && re.a_rows != nullptr && m0 + r < m_end) ? re.a_rows[m0 + r] : m0 + r;
        voff[h][i] = h < 2 ? (m0 + r < m_end ? (uint32_t)((size_t)arow * lda * 2) + ch * 16 : 0x80000000u)
                           : (uint32_t)((size_t)min(n0 + r, N - 1) * ldb * 2) + ch * 16;
      }
    auto issue_half = [&](int buf, int h, int kt) {
      const uint32_t soff = (uint32_t)(k0 + kt) * kBK * 2;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int r0 = h < 2 ? i * 128 + h * 64 + wid * 8 : (h & 1) * 128 + (wid + 8 * i) * 8;
        uint16_t* dst = smem + buf * BUF + (h >= 2 ? BM * kBK : 0) + r0 * kBK;
        if (GROUPED && h >= 2 && re.b_nt && b_once)  // an expert's weights streamed once
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_void_t*)dst, 16, voff[h][i], soff, 0, 2 /* nt */);
        else
          __builtin_amdgcn_raw_ptr_buffer_load_lds(h < 2 ? rsA : rsB, (lds_void_t*)dst, 16, voff[h][i], soff, 0, 0);
      }
    };
    auto read_a = [&](int buf, int mi, bf16x8 (&fa)[4][2]) {
      const uint16_t* sA = smem + buf * BUF;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = grp * 128 + mi * 64 + i * 16 + (lane & 15);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const int ch = kk * 4 + (lane >> 4);
          fa[i][kk] = *reinterpret_cast<const bf16x8*>(sA + r * kBK + ((ch ^ swz(r)) << 3));
        }
      }
    };
    auto read_b = [&](int buf, int nj, bf16x8 (&fb)[2][2]) {
      const uint16_t* sB = smem + buf * BUF + BM * kBK;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = wc * 64 + nj * 32 + j * 16 + (lane & 15);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const int ch = kk * 4 + (lane >> 4);
          fb[j][kk] = *reinterpret_cast<const bf16x8*>(sB + r * kBK + ((ch ^ swz(r)) << 3));
        }
      }
    };

#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // a 64-row quadrant wholly past the tile's last row issues no MFMAs (wave-uniform): the
    // partner group's MFMAs then run alone on the SIMD.  Ragged M, and above all the last
    // m-tile of every expert in the grouped (MoE) GEMM, half empty on average.
    const int rows_here = sk.skip_dead ? m_end - m0 : BM;
    // K-loop: two phases per K-tile, 32 MFMAs each.
    //   X(t): read A(mi 0) + B(nj 0, 1) of t | DMA A(mi 1) of t+1 -> buffer (t+1)&1
    //   Y(t): read A(mi 1) of t             | DMA A(mi 0) + B of t+2 -> buffer t&1
    // Group 1 runs one barrier behind group 0, so each SIMD's two waves alternate: one issues
    // its phase's LDS reads and DMAs while the other runs 32 MFMAs.  (The guide's 4 x 16-MFMA
    // template hands the matrix core over twice as often: 2-9 % slower on every Llama-3-8B
    // projection, profiles/r03_gemm_fourwave.md.)  Every phase drains its LDS reads before its
    // first barrier, so a buffer region can be restaged in the phase after its last read; every
    // wait (counted vmcnt) precedes the first barrier of the phase before the reads (RAW across
    // the staggered groups):
    //   X(t) wait: A(mi 1, t) retired; 8 younger DMAs (A0+B of t+1, A1 of t+1) stay in flight
    //   Y(t) wait: A(mi 0) + B of t+1 retired; A1(t+1) and A0+B(t+2) stay in flight
    bf16x8 fa[4][2], fb0[2][2], fb1[2][2];
    auto seg_mma = [&](int mi) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // drain before the barrier
      raw_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // a 64-row quadrant wholly past the tile's last row issues no MFMAs (wave-uniform)
      if (grp * 128 + mi * 64 < rows_here) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          // balance 2: 16-row blocks past the last row skipped too (wave-uniform; a 257-row
          // expert's balanced tiles then do 8 and 9 blocks, near-equal, and stay in step)
          if (i > 0 && sk.balance == 2 && grp * 128 + mi * 64 + i * 16 >= rows_here) continue;
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
              acc[mi * 4 + i][j] = mfma16(fa[i][kk], fb0[j][kk], acc[mi * 4 + i][j]);
              acc[mi * 4 + i][2 + j] = mfma16(fa[i][kk], fb1[j][kk], acc[mi * 4 + i][2 + j]);
            }
        }
        __builtin_amdgcn_s_setprio(0);
      }
      __builtin_amdgcn_sched_barrier(0);
      raw_barrier();
    };
    issue_half(0, 0, 0);
    issue_half(0, 1, 0);
    issue_half(0, 2, 0);
    issue_half(0, 3, 0);
    if (nkp > 1) { issue_half(1, 0, 1); issue_half(1, 2, 1); issue_half(1, 3, 1); }
    if (nkp > 1) wait_vmcnt<6>(); else wait_vmcnt<0>();
    raw_barrier();
    if (grp == 1) raw_barrier();  // stagger: group 1 runs one barrier behind group 0
    for (int t = 0; t < nkp; ++t) {
      const int cur = t & 1, nxt = cur ^ 1;
      const bool m1 = t + 1 < nkp, m2 = t + 2 < nkp;
      read_a(cur, 0, fa);  // X(t)
      read_b(cur, 0, fb0);
      read_b(cur, 1, fb1);
      if (m1) {
        issue_half(nxt, 1, t + 1);
        wait_vmcnt<8>();
      } else {
        wait_vmcnt<0>();
      }
      seg_mma(0);
      read_a(cur, 1, fa);  // Y(t)
      if (m2) {
        issue_half(cur, 0, t + 2);
        issue_half(cur, 2, t + 2);
        issue_half(cur, 3, t + 2);
        wait_vmcnt<8>();
      } else if (m1) {
        wait_vmcnt<2>();
      }
      seg_mma(1);
    }
    if (grp == 0) raw_barrier();  // barrier counts of the two groups must match
    __syncthreads();              // all LDS reads retired everywhere: the ring becomes C staging

    if (SK && k1 - k0 != nk) {
      // stream-K partial tile: slot, ticket, and (last contributor only) the fixup
      const int s = s_idx, base = t0 * nk;
      auto slot_of = [&](int w) { return 2 * w + (tile == (base + w * ipw) / nk ? 0 : 1); };
      const int first_w = (tile * nk - base) / ipw, last_w = (tile * nk + nk - 1 - base) / ipw;
      // hand-off (MI355X_MICROARCH.md "Valid forms", first table row): 16-B sc1 (write-through)
      // stores, every storing wave's vmcnt(0), a barrier, ONE lane's agent-scope ticket add;
      // the workgroup whose add came last loads the other slots with 16-B sc1 loads after a
      // barrier.  No L2 write-back / invalidate: an agent release here (buffer_wbl2) writes
      // back every dirty line of the XCD's L2 -- the C tiles of the other workgroups too.
      constexpr int kSlotBytes = BM * BN * 4;
      auto slot_rsrc = [&](int w) {
        return __builtin_amdgcn_make_buffer_rsrc(sk.ws + (size_t)slot_of(w) * (BM * BN), 0, kSlotBytes, 0x00020000);
      };
      {
        const auto rs = slot_rsrc(s);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs, tid * 16,
                                                   (i * 4 + j) * 512 * 16, 16 /* sc1 */);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      int* flag = reinterpret_cast<int*>(smem);
      if (tid == 0) {
        const int t = __hip_atomic_fetch_add(sk.cnt + (tile - t0), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool last = t == last_w - first_w;
        if (last) __hip_atomic_store(sk.cnt + (tile - t0), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        flag[0] = last;
      }
      __syncthreads();
      const int last = flag[0];
      __syncthreads();  // flag read everywhere before the epilogue reuses the LDS
      if (!last) continue;
      // deterministic sum: with 2 contributors own + other is exact whichever arrives last;
      // with 3+ the last one re-reads its own slot and sums every slot in contributor order
      const bool reload = last_w - first_w >= 2;
      if (reload) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      for (int w = first_w; w <= last_w; ++w) {
        if (w == s && !reload) continue;
        const auto rs = slot_rsrc(w);
        // 16 loads in flight per batch: one load -> wait -> add at a time is ~1.5 us per
        // round trip, 48 us per slot (the compiler keeps these loads in program order)
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          f32x4 v[16];
#pragma unroll
          for (int q = 0; q < 16; ++q)
            v[q] = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, tid * 16, (g * 16 + q) * 512 * 16, 16 /* sc1 */));
#pragma unroll
          for (int q = 0; q < 16; ++q) acc[(g * 16 + q) / 4][q % 4] += v[q];
        }
      }
    }

    if constexpr (EPI == EPI_ROPE) {
      // stage the whole 256 x 256 bf16 tile (two heads), then rotate / scatter per head
      constexpr int LDR = BN + 8;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = grp * 128 + i * 16 + 4 * (lane >> 4) + r;
#pragma unroll
          for (int j = 0; j < 4; ++j) smem[row * LDR + wc * 64 + j * 16 + (lane & 15)] = f2bf(acc[i][j][r]);
        }
      __syncthreads();
      const int rows = min(BM, m_end - m0);
      auto at = [&](int r, int c) { return bf2f(smem[r * LDR + c]); };
      rope_tile_store<512>(at, n0 / 128, 2, m0, rows, re, tid);
      continue;
    }
    // epilogue: each wave stages its 128 x 64 (or 128 x 32 after SiLU.mul) bf16 tile
    constexpr int OW = EPI == EPI_NONE ? 64 : 32;
    constexpr int LD = OW + 8;
    uint16_t* sC = smem + wid * 128 * LD;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = i * 16 + 4 * (lane >> 4) + r;
        if constexpr (EPI == EPI_NONE) {
#pragma unroll
          for (int j = 0; j < 4; ++j) sC[row * LD + j * 16 + (lane & 15)] = f2bf(acc[i][j][r]);
        } else {
#pragma unroll
          for (int jp = 0; jp < 2; ++jp) {
            const float g = acc[i][2 * jp][r], u = acc[i][2 * jp + 1][r];
            sC[row * LD + jp * 16 + (lane & 15)] = f2bf(silu_bf(g) * bf2f(f2bf(u)));
          }
        }
      }
    __syncthreads();
    constexpr int CPR = OW / 8;  // 16-B chunks per staged row
    const int out_col0 = EPI == EPI_NONE ? n0 + wc * 64 : (n0 + wc * 64) / 2;
    const int out_n = EPI == EPI_NONE ? N : N / 2;
#pragma unroll
    for (int i2 = 0; i2 < 128 * CPR / 64; ++i2) {
      const int c = i2 * 64 + lane;
      const int row = c / CPR, cc = (c % CPR) * 8;
      const int gm = m0 + grp * 128 + row, gn = out_col0 + cc;
      if (gm < m_end && gn < out_n) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(sC + row * LD + cc);
        if (re.ws_nt & 4) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(C + (size_t)gm * ldc + gn));
        else *reinterpret_cast<u32x4*>(C + (size_t)gm * ldc + gn) = v;
      }
    }
  } while (SK && it < it_end);
}

// Stream-K buffers (per device, allocated once outside graph capture by gemm_sk_reserve):
// 2 partial slots per stream-K workgroup and kCntRegions rotating sets of tail-tile counters,
// so back-to-back launches never share a counter set while one may still be resetting.
constexpr int kSkMaxWg = 256, kCntRegions = 64;
struct SkBuf {
  float* ws = nullptr;
  int* cnt = nullptr;
  int next = 0, cus = 0;
};
static SkBuf g_sk[16];
static int g_sk_mode = 1;
static const int g_sk_min_iters = 16;
static const int g_skip_dead = 1;
// gemm_grouped_balance op: 1 = quadrant-aligned equal row ranges for an expert over several
// m-tiles (8 x 257 rows gate_up 677 -> 639 us, down 353 -> 308; Mixtral batch 1024 +0.75 %);
// 2 (default) = that + 16-row blocks past the tile's last row skip their MFMAs, so the two
// tiles of a 257-row expert do 8 and 9 blocks (gate_up 597 us; batch 1024 +0.3-0.5 % over 1)
// (profiles/r06_moe_spill.md)
static int g_grouped_balance = 2;
int gemm_grouped_balance(int set) {
  if (set >= 0) g_grouped_balance = set;
  return g_grouped_balance;
}
static int g_grouped_order = 2;  // 0 slot fastest, 1 expert-major, 2 expert-major from 3 m-tiles / expert
int gemm_grouped_order(int set) {
  if (set >= 0) g_grouped_order = set;
  return g_grouped_order;
}

int gemm_sk_mode(int set) {
  if (set >= 0) g_sk_mode = set;
  return g_sk_mode;
}

bool gemm_sk_reserve() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return false;
  SkBuf& b = g_sk[dev];
  if (b.ws) return true;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) return false;
  b.cus = std::min(cus, kSkMaxWg);
  float* ws = nullptr;
  int* cnt = nullptr;
  if (hipMalloc((void**)&ws, (size_t)2 * kSkMaxWg * 256 * 256 * sizeof(float)) != hipSuccess) return false;
  if (hipMalloc((void**)&cnt, (size_t)kCntRegions * kSkMaxWg * sizeof(int)) != hipSuccess) {
    (void)hipFree(ws);
    return false;
  }
  if (hipMemset(cnt, 0, (size_t)kCntRegions * kSkMaxWg * sizeof(int)) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    (void)hipFree(ws);
    (void)hipFree(cnt);
    return false;
  }
  b.ws = ws;
  b.cnt = cnt;
  return true;
}

// Split of a plain launch's T tiles: n_dp data-parallel workgroups + a stream-K tail
// (n_sk = 0: no tail).  The r = T % C tail tiles are each cut into d equal K-ranges (d | nk,
// so no range straddles two tiles), one per extra workgroup, d <= C / r, when the cost model
// (in K-tile times, calibrated on scripts/bench_proj.py) beats the tail round's nk:
//   ipw                      the range itself
//   max(2, w * 0.04)         256 KB fp32 partial per workgroup, HBM-bound when all write
//   (d - 1 or d) * 2         the last contributor's slot reads (one CU, ~3 us per slot)
//   1                        a second pipeline fill + ticket
// Ranges that straddle tiles (general stream-K) were measured slower than the data-parallel
// grid whenever the tail exceeds half the chip: twice the partial traffic, two fills.
static int sk_min_half() { return std::max(1, g_sk_min_iters / 2); }

static SkBuf* sk_buf() {
  int dev = 0;
  if (!g_sk_mode || hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return nullptr;
  SkBuf& b = g_sk[dev];
  return b.ws && b.cus > 0 ? &b : nullptr;
}

// partial-tile scratch for the four-wave kernel's split tail (gemm_w4.hip): the same per-device
// slot buffer and a rotated ticket-counter region; false when the buffers are not reserved
bool gemm_sk_scratch(float** ws, int** cnt, int* cus) {
  SkBuf* b = sk_buf();
  if (!b) return false;
  *ws = b->ws;
  *cnt = b->cnt + (size_t)(b->next++ % kCntRegions) * kSkMaxWg;
  *cus = b->cus;
  return true;
}

bool gemm_sk_available(int* cus) {
  SkBuf* b = sk_buf();
  if (b && cus) *cus = b->cus;
  return b != nullptr;
}

static SkArgs sk_plan(int T, int nk, int& n_sk) {
  SkArgs a{T, T, 1, 0, nullptr, nullptr, T, 256, sk_min_half(), g_skip_dead};
  n_sk = 0;
  SkBuf* b = sk_buf();
  if (!b) return a;
  const int d = sk_choose_d(T, nk, b->cus, sk_min_half());
  if (!d) return a;
  const int r = T % b->cus;
  a.n_dp = T - r;
  a.t0 = T - r;
  a.ipw = nk / d;
  a.n_iters = r * nk;
  a.ws = b->ws;
  a.cnt = b->cnt + (size_t)(b->next++ % kCntRegions) * kSkMaxWg;
  a.n_base = a.n_dp;
  a.cus = b->cus;
  n_sk = r * d;
  return a;
}

template <int EPI, bool GROUPED = false>
static void run_pp(const uint16_t* A, int lda, const uint16_t* B, int ldb, uint16_t* C, int ldc, int M,
                   int N, int K, hipStream_t st, const RopeEpi& re, const int* offsets = nullptr,
                   int n_groups = 0) {
  constexpr size_t ring = 2ull * (256 + 256) * kBK * 2;
  constexpr size_t epi = EPI == EPI_ROPE ? 256ull * (256 + 8) * 2
                                         : 8ull * 128 * ((EPI == EPI_NONE ? 64 : 32) + 8) * 2;
  constexpr size_t lds = ring > epi ? ring : epi;
  static_assert(lds <= 163840, "LDS budget");
  auto kern = gemm_pp_kernel<EPI, GROUPED>;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int gx = (N + 255) / 256, gy = (M + 255) / 256 + (GROUPED ? n_groups : 0);
  constexpr int group_m = 4;
  const int gm = std::max(1, std::min(group_m, gy));
  int n_sk = 0;
  SkArgs sk = sk_plan(gx * gy, K / kBK, n_sk);
  // expert weights non-temporal where the expert fits one 256-row m-tile (decided per tile on
  // device): Mixtral batch 256 (64 rows per expert on average) +3.9 %; nt on every expert lost
  // 1.5 % at batch 1024, where the spill m-tiles of the > 256-row experts re-read the weights
  RopeEpi r = re;
  r.b_nt = GROUPED && (g_small_nt_flags & 4) != 0;
  r.ws_nt = g_slab_nt;
  if constexpr (GROUPED) {
    // the routed tile count is only known on device: the grid is the worst case (every
    // expert's last m-tile partial) plus one stream-K block per CU; the kernel plans the
    // split from offsets[] with the same sk_choose_d and idles the blocks it does not need
    SkBuf* b = sk_buf();
    const int T_max = gx * gy;
    sk = SkArgs{T_max, T_max, 1, 0, nullptr, nullptr, T_max, 256, sk_min_half(), g_skip_dead, g_grouped_balance, g_grouped_order};
    if (b) {
      sk.ws = b->ws;
      sk.cnt = b->cnt + (size_t)(b->next++ % kCntRegions) * kSkMaxWg;
      sk.cus = b->cus;
      n_sk = b->cus;
    }
  }
  if (n_sk > 0) {
    auto ksk = gemm_pp_kernel<EPI, GROUPED, true>;
    static bool attr_sk = false;
    if (!attr_sk) {
      hipFuncSetAttribute((const void*)ksk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      attr_sk = true;
    }
    ksk<<<sk.n_base + n_sk, 512, lds, st>>>(A, lda, B, ldb, C, ldc, M, N, K, gx, gy, gm, r, offsets, n_groups, sk);
    return;
  }
  kern<<<gx * gy, 512, lds, st>>>(A, lda, B, ldb, C, ldc, M, N, K, gx, gy, gm, r, offsets, n_groups, sk);
}

struct Plan {
  int BM, BN, splits, k_chunk, m_tiles, variant;
  int stages;  // LDS-DMA ring depth of the small-M tiles (0: g_small_stages)
  bool nosplit;  // grouped: one K range (the mid-size MoE split-K below is skipped)
};


// Tile choice by the (per-group) row count:
//   M <= 64 / 128: narrow tiles, many WGs (weight streaming);  M <= 256: the whole
//   batch in one tile (weights read once), BN by how many N tiles fill the chip;
//   large M: variant 0 = 256x128 (3-stage ring), 1 = 256x256 (2-stage, 128x64 per
//   wave: half the LDS + L2 bytes per FLOP), 2 = 256x256 + setprio around MFMAs,
//   3 = 256x256 two-group ping-pong (gemm_pp_kernel), 5 (default) = the four-wave kernel with
//   the hand-scheduled asm K-loop (gemm_w4.hip) where its grid fills the chip, else 3.  (A four-wave 128x128-per-wave
//   variant was measured 10-20% slower: profiles/r02_gemm_fourwave_rejected.md.)
// true when the stream-K tail is available here and splits ALL T (<= C / 2) tiles
static bool sk_halves_ok(long T, int nk) {
  const SkBuf* b = sk_buf();
  return b && T * 2 <= b->cus && sk_choose_d((int)T, nk, b->cus, sk_min_half()) >= 2;
}

static Plan plan(int M, int N, int K, bool grouped, int n_groups, int rows_per_group) {
  Plan p{};
  p.variant = 0;
  const int mrows = grouped ? rows_per_group : M;
  // grouped (MoE): the ping-pong kernel from ~56 routed rows per expert.  Its 256 x 256 tile
  // streams each expert's weight panel once per n-tile and skips the MFMAs of empty 64-row
  // quadrants, so a half-empty expert tile costs less than the extra m-tiles (each a second walk
  // of the expert's weights) of the narrower kernels: Mixtral gate_up / down at 512 routed rows
  // 474 -> 370 / 266 -> 200 us, 1024 rows 692 -> 389 / 375 -> 208 us; 48 rows per expert equal
  // (scripts/bench_moe_decode.py, profiles/r05_moe_decode.md)
  constexpr int pp_group_min_rows = 56;
  if (grouped && mrows >= pp_group_min_rows && K % kBK == 0 && N % 256 == 0) {
    p.BM = 256; p.BN = 256; p.variant = 3;  // grouped ping-pong
  } else if (mrows <= 64 && !grouped && g_small_tile == 1) {
    // per shape (scripts/run137.sh, cold us at M = 16): wide N (gate_up) 64 columns with a
    // 6-deep ring (47.0 -> 44.8); narrow N 32 columns with an 8-deep ring at BM 16 (qkv
    // 15.3 -> 13.5, o / down unchanged): more weight bytes in flight per CU
    p.BM = mrows <= 16 ? 16 : mrows <= 32 ? 32 : 64;
    p.BN = 64;
    // (M 17-32 narrow projections on the 32-column 8-deep tiles of M <= 16: 1-2 % slower end to
    // end at batch 24 / 32, scripts/history INDEX run140)
    if (p.BM == 16) {
      const bool wide = N >= 16384;
      p.BN = wide ? 64 : 32;
      p.stages = wide ? (p.BM == 16 ? 6 : 0) : 8;
    } else if (p.BM == 64) {
      // M 33-64: narrow N on the 6-deep ring (run133: qkv 19.8 -> 18.4, down+norm 35.9 -> 32.0 us),
      // gate_up on a 4-deep one (run145: 48.2 -> 47.1 at M = 64, 6 stages lose: 50.4)
      p.stages = N < 16384 ? 6 : 4;
    }
  } else if (mrows <= 64 && !grouped && (g_small_tile == 32 || g_small_tile == 64)) {
    p.BM = mrows <= 16 ? 16 : mrows <= 32 ? 32 : 64;
    p.BN = g_small_tile;
  } else if (mrows <= 64) {
    p.BM = 64;
    p.BN = 64;
    // grouped (MoE at a few dozen rows per expert), narrow down projection: ring depth knob
    if (grouped && N < 16384) p.stages = g_grouped_small_stages;
    // grouped at <= 32 rows per expert (Mixtral batch 16-64): down on 32 x 64 tiles with a
    // 6-deep ring and ONE K range, gate_up on a 4-deep ring (scripts/bench_moe_decode.py, cold
    // expert weights, profiles/r05_moe_decode.md: down at 128 routed rows 172.4 -> 160.4 us,
    // 5.45 -> 5.86 TB/s; gate_up 318.2 -> 315.9)
    if (grouped && g_grouped_narrow && mrows <= 32) {
      if (N < 16384) { p.BM = 32; p.stages = 6; p.nosplit = true; }
      else p.stages = 4;
    }
  }
  else if (mrows <= 128) { p.BM = 128; p.BN = 64; }
  else if (mrows <= 256) {
    constexpr int bn_min_tiles = 192;
    p.BM = 256;
    p.BN = ((N + 127) / 128 >= bn_min_tiles) ? 128 : 64;
  } else {
    const int big = g_big_variant;
    constexpr int big_min_m = 1024;
    p.BM = 256;
    p.BN = 128;
    // 128: o / down at 2049-2816 rows (the mixed steps of batch ~512: 144-176 tiles, no K-half
    // tail for the four-wave kernel) ran on the 256 x 128 kernel at 0.55x hipBLASLt; the
    // ping-pong kernel's stream-K tail takes them (o at M = 2560: 122 -> 88 us, down 394 -> 269;
    // scripts/history/r4_m2560.sh)
    constexpr int pp_min_tiles = 128;
    const long t256 = (long)((M + 255) / 256) * ((N + 255) / 256);
    // below pp_min_tiles the 256x256 grid leaves CUs idle, unless the stream-K tail can cut
    // every tile in two (T <= C / 2): o / down at M = 2040 (128 tiles)
    const bool pp_ok = K % kBK == 0 && (t256 >= pp_min_tiles || sk_halves_ok(t256, K / kBK));
    // variant 5: the four-wave kernel where its grid fills the chip: >= w4_min_tiles tiles, or
    // a tail it can cut in K-halves (o / down at M = 2048: 128 tiles -> 256 half-tiles); else
    // the ping-pong kernel with its general stream-K tail
    constexpr int w4_min_tiles = 192;
    const bool w4_fills = t256 >= w4_min_tiles || gemm_w4_split_ok((int)t256, K / kBK);
    // Wide projections take the large-M kernels from 512 rows: gate_up / lm_head at M = 512 /
    // 768 ran 127 -> 87 / 191 -> 153 us (8B) and 511 -> 404 us (70B gate_up), batch-512 serving
    // +5.3 %; narrow ones lose there (o / down at M = 512: 31 -> 48 / 66 -> 124 us) and keep the
    // 256 x 128 kernel (scripts/history/r4_bigminm.sh, r4_bigminm2.sh, r4_widemin.sh).
    // Below ~72 tiles of 256 x 256 (o / down at M = 512 - 1024: 32 - 64 tiles) the 256 x 128
    // kernel beats them at every M measured short of 2048 (o at M = 1024: 44.7 vs 48.6 us, down
    // 114.7 vs 129.5); from 72 tiles (qkv at M = 768, 70B qkv at 512) the large-M kernels win.
    constexpr int wide_min_m = 512;
    constexpr int mid_tiles = 72;
    const int big_from = t256 >= mid_tiles ? std::min(big_min_m, wide_min_m) : std::max(big_min_m, 2048);
    if (big == 5 && !(mrows >= big_from && !grouped && w4_fills && gemm_w4_ok(M, N, K, K, K))) {
      if (mrows >= big_from && !grouped && pp_ok) { p.BN = 256; p.variant = 3; }
    } else if (big && mrows >= big_from && !grouped && (big < 3 || pp_ok)) {
      p.BN = 256;
      p.variant = big;
    }
    if (!grouped && big == 5) {
      // long-K narrow projections (down, K = 14336) at 40-71 tiles of 256 x 256 (M 640-1279):
      // the ping-pong kernel's stream-K tail spreads the few tiles' K over every CU (down at
      // M = 768: 105 -> 90 us, 1024: 118 -> 108; hipBLASLt 90 / 111)
      if (p.variant == 0 && K >= 8192 && t256 >= 40 && t256 < mid_tiles && K % kBK == 0 &&
          sk_halves_ok(t256, K / kBK)) {
        p.BN = 256;
        p.variant = 3;
      }
      // four-wave vs ping-pong past one full round: the four-wave kernel runs whole rounds of
      // 256 x 256 tiles (a tail of r <= CUs / 2 tiles in K-halves), the ping-pong kernel ~7 %
      // slower per tile but with a stream-K tail that balances ANY remainder.  Estimated time in
      // four-wave tile rounds: w4 = q + (r ? (2r <= C ? 0.55 : 1) : 0), pp = 1.08 T / C + 0.05.
      // (M = 4608: o 147 -> 134 us, down 476 -> 403, qkv 181 -> 172; the headline's M ~ 4088 is
      // whole rounds for every projection and stays on the four-wave kernel; bench_mid_m.py)
      const SkBuf* b = sk_buf();
      if (p.variant == 5 && b && t256 > b->cus && pp_ok) {
        const long C = b->cus, q = t256 / C, r = t256 % C;
        const float w4_est = (float)q + (r == 0 ? 0.f : (2 * r <= C ? 0.55f : 1.f));
        const float pp_est = 1.08f * (float)t256 / (float)C + 0.05f;
        if (pp_est < w4_est - 0.03f) p.variant = 3;
      }
      // variant 6, the half-height (128 x 256) four-wave tile, where its grid is at most one
      // round: up to twice the workgroups of the 256 x 256 grid (a lone tile of either height
      // runs ~1.8x faster than one in a full round, so idle CUs cost more than the half tile's
      // lower MFMA density).  bench_mid_m.py (profiles/r05_gemm_w4h.md), planner before -> after:
      // o at M = 1024 / 1536 / 2048 46.2 -> 38.3 / 56.0 -> 47.6 / 65.6 -> 55.2 us, qkv at 384 /
      // 512 / 1024 43.1 -> 33.1 / 44.4 -> 35.3 / 56.0 -> 47.5; past one round it loses to the
      // full tile (qkv 1408: 75.9 vs 72.3).  Long K (down): only with its own K-half tail
      // (t128 <= CUs / 2: 96 -> 256 items, M = 1024 110.8 -> 98.5); without it the full tile's
      // K-halves win (M = 1152: 153.7 vs 131.1), and below ~80 tiles the 256 x 128 split-K kernel
      // (M = 512: 83.1 vs 67.6).
      const long t128 = (long)((M + 127) / 128) * ((N + 255) / 256);
      const bool long_k = K >= 8192;
      if (g_half_tile && b && mrows >= 384 && (long_k ? t128 >= 80 && 2 * t128 <= b->cus : t128 >= 64 && t128 <= b->cus) &&
          (p.variant == 0 || p.variant == 3 || p.variant == 5) && gemm_w4_ok(M, N, K, K, K)) {
        p.BM = 128;
        p.BN = 256;
        p.variant = 6;
      }
    }
  }
  if (!grouped && g_dp[0] >= 0) {  // bench override (gemm_dense_plan)
    p.variant = g_dp[0];
    p.BM = p.variant == 0 ? g_dp[1] : p.variant == 6 ? 128 : 256;
    p.BN = p.variant == 0 ? g_dp[2] : 256;
    p.stages = g_dp[4];
  }
  if (grouped && g_gp[0] > 0) {  // bench override (gemm_grouped_plan)
    p.BM = g_gp[0];
    p.BN = g_gp[1];
    p.variant = (p.BM == 256 && p.BN == 256) ? 3 : 0;
    p.stages = g_gp[2] > 0 ? g_gp[2] : 0;
  }
  const int n_tiles = (N + p.BN - 1) / p.BN;
  const int real_m_tiles = (M + p.BM - 1) / p.BM;
  p.m_tiles = grouped ? real_m_tiles + n_groups : real_m_tiles;
  p.splits = 1;
  p.k_chunk = K;
  const long tiles = (long)n_tiles * real_m_tiles;
  // run49: down -5..-15% at M 8-64.  The 16-row tiles (M 9-16) aim at 512 workgroups: batch 16
  // +5.6 / +6.0 % interleaved (scripts/r5_splittarget.sh, r5_splittarget2.sh), while 512 lost
  // 1.4-1.6 % at batch 24 / 32 (32-row tiles), 5 % at batch 64 and 4 % at 256
  const int split_target = p.BM <= 16 ? g_split_target : 256;
  constexpr int split_max_tiles = 160;
  if (!grouped && tiles < split_max_tiles && K >= 1024 && p.variant != 3 && p.variant < 5) {
    int s = (int)std::min<long>(8, std::max<long>(1, split_target / tiles));
    int kc = ((K / s + kBK - 1) / kBK) * kBK;
    p.splits = (K + kc - 1) / kc;
    p.k_chunk = kc;
  }
  if (!grouped && g_dp[0] == 0 && g_dp[3] >= 1) {
    const int kc = ((K / g_dp[3] + kBK - 1) / kBK) * kBK;
    p.splits = (K + kc - 1) / kc;
    p.k_chunk = kc;
  }
  return p;
}

template <int EPI, bool GROUPED>
static void launch_plan(const Plan& p, const uint16_t* A, int lda, const uint16_t* B, int ldb,
                        uint16_t* C, int ldc, float* ws, int M, int N, int K, const int* offsets,
                        int n_groups, hipStream_t st, const RopeEpi& re = RopeEpi{}) {
#define MLOP_GEMM(bm, bn, wm, wn, stages, prio)                                                   \
  run_cfg<bm, bn, wm, wn, EPI, GROUPED, stages, prio>(A, lda, B, ldb, C, ldc, ws, M, N, K,        \
                                                      p.splits, p.k_chunk, offsets, n_groups,     \
                                                      p.m_tiles, st, re)
  if constexpr (EPI == EPI_ROPE) {  // whole heads per staged chunk, no split-K (launch_gemm_rope)
    if (p.BN == 128) MLOP_GEMM(256, 128, 4, 2, 3, false);
    else if (!GROUPED && p.variant >= 5 && gemm_w4_ok(M, N, K, lda, ldb, ldc))
      run_w4(EPI, A, lda, B, ldb, C, ldc, M, N, K, st, re, p.BM);
    else if (!GROUPED && (p.variant == 3 || p.variant >= 5)) run_pp<EPI>(A, lda, B, ldb, C, ldc, M, N, K, st, re);
    else if (!GROUPED && p.variant == 2) MLOP_GEMM(256, 256, 2, 4, 2, true);
    else if (!GROUPED) MLOP_GEMM(256, 256, 2, 4, 2, false);
  } else {
    // weight-streaming tiles (M <= 128): a deeper LDS-DMA ring keeps more weight bytes in
    // flight per CU (3 stages x 16 KB per workgroup streamed gate_up at 4.7 TB/s at M = 64)
    const int sst = p.stages ? p.stages : g_small_stages;
    if (!GROUPED && p.variant == 6 && p.splits == 1 && gemm_w4_ok(M, N, K, lda, ldb, ldc))
      run_w4(EPI, A, lda, B, ldb, C, ldc, M, N, K, st, re, 128);
    else if (!GROUPED && p.variant == 6) run_pp<EPI>(A, lda, B, ldb, C, ldc, M, N, K, st, re);
    else if (p.BM == 16 && p.BN == 32 && sst >= 8) MLOP_GEMM(16, 32, 1, 2, 8, false);
    else if (p.BM == 16 && p.BN == 32 && sst >= 6) MLOP_GEMM(16, 32, 1, 2, 6, false);
    else if (p.BM == 16 && p.BN == 32) MLOP_GEMM(16, 32, 1, 2, 4, false);
    else if (p.BM == 16 && p.BN == 64 && sst >= 8) MLOP_GEMM(16, 64, 1, 2, 8, false);
    else if (p.BM == 16 && p.BN == 64 && sst >= 6) MLOP_GEMM(16, 64, 1, 2, 6, false);
    else if (p.BM == 16 && p.BN == 64) MLOP_GEMM(16, 64, 1, 2, 4, false);
    else if (p.BM == 32 && p.BN == 32 && sst >= 8) MLOP_GEMM(32, 32, 1, 2, 8, false);
    else if (p.BM == 32 && p.BN == 32) MLOP_GEMM(32, 32, 1, 2, 4, false);
    else if (p.BM == 32 && p.BN == 64 && sst >= 6) MLOP_GEMM(32, 64, 1, 4, 6, false);
    else if (p.BM == 32 && p.BN == 64) MLOP_GEMM(32, 64, 1, 4, 4, false);
    else if (p.BM == 64 && p.BN == 32) MLOP_GEMM(64, 32, 1, 2, 4, false);
    else if (p.BM == 64 && p.BN == 64 && sst >= 6) MLOP_GEMM(64, 64, 1, 4, 6, false);
    else if (p.BM == 64 && p.BN == 64 && sst == 4) MLOP_GEMM(64, 64, 1, 4, 4, false);
    else if (p.BM == 64) MLOP_GEMM(64, 64, 1, 4, 3, false);
    else if (p.BM == 128 && g_small_stages >= 5) MLOP_GEMM(128, 64, 2, 2, 5, false);
    else if (p.BM == 128) MLOP_GEMM(128, 64, 2, 2, 3, false);
    else if (p.BN == 64) MLOP_GEMM(256, 64, 4, 2, 3, false);
    else if (p.BN == 128) MLOP_GEMM(256, 128, 4, 2, 3, false);
    else if (GROUPED && p.variant == 3)
      run_pp<EPI, true>(A, lda, B, ldb, C, ldc, M, N, K, st, re, offsets, n_groups);
    else if (!GROUPED && p.variant == 5 && p.splits == 1 && gemm_w4_ok(M, N, K, lda, ldb, ldc))
      run_w4(EPI, A, lda, B, ldb, C, ldc, M, N, K, st, re);
    else if (!GROUPED && (p.variant == 3 || p.variant == 5) && p.splits == 1)
      run_pp<EPI>(A, lda, B, ldb, C, ldc, M, N, K, st, re);
    else if (!GROUPED && p.variant == 2) MLOP_GEMM(256, 256, 2, 4, 2, true);
    else if (!GROUPED) MLOP_GEMM(256, 256, 2, 4, 2, false);
  }
#undef MLOP_GEMM
}

// stream-K workgroups a plain launch of this shape would add (0: data-parallel grid only)
int gemm_sk_workgroups(int M, int N, int K) {
  if (M <= 0 || gemv_takes(M, N, K, EPI_NONE)) return 0;
  const Plan p = plan(M, N, K, false, 0, 0);
  if (p.variant != 3 || p.BN != 256 || p.splits != 1) return 0;
  int n_sk = 0;
  sk_plan(((M + 255) / 256) * ((N + 255) / 256), K / kBK, n_sk);
  return n_sk;
}

// EPI_ROPE: the plain (no split-K) plan must stage whole heads: BN >= 128, i.e. M > 256.
// Small M whose plan splits K: the slabs go to the stream-K scratch and the split-K reduce is
// fused into the RoPE + cache kernel (one launch instead of reduce + rope_cache).
static bool rope_slabs_ok(const Plan& p, int M, int N) {
  const SkBuf* b = sk_buf();
  return p.splits > 1 && p.variant != 3 && p.variant < 5 && b != nullptr &&
         (size_t)p.splits * M * N <= (size_t)2 * kSkMaxWg * 256 * 256;
}

// Small-M QKV: K split even where the plain plan keeps one K range (M <= 16: 192 tiles of 16 x
// 32): the slabs' reduce rides in the RoPE + cache kernel that runs anyway, so a second K range
// costs one fp32 slab and doubles the workgroups streaming the weights (gemm_rope_split op:
// the K ranges, 1 = the plain plan).  Interleaved, scripts/r5_ropesplitk.sh: batch 16 +1.9 %,
// batch 12 +3.0 % (4 ranges: +2.2 / +2.6 %)
static int g_rope_split_k = 2;
int gemm_rope_split(int set) {
  if (set >= 1) g_rope_split_k = set;
  return g_rope_split_k;
}

static Plan rope_plan(int M, int N, int K) {
  Plan p = plan(M, N, K, false, 0, 0);
  if (g_rope_split_k > 1 && p.splits == 1 && p.variant == 0 && p.BM <= 64 && K >= 2048) {
    const int kc = ((K / g_rope_split_k + kBK - 1) / kBK) * kBK;
    p.splits = (K + kc - 1) / kc;
    p.k_chunk = kc;
  }
  return p;
}

bool gemm_rope_supported(int M, int N, int K) {
  if (M <= 0 || N % 128 || K % kBK) return false;
  if (gemv_takes(M, N, K, EPI_ROPE)) return true;  // decode M <= 8: gemv.hip
  const Plan p = rope_plan(M, N, K);
  return ((p.BM == 256 || p.variant == 6) && p.BN >= 128) || rope_slabs_ok(p, M, N);
}

bool launch_gemm_rope(const void* A, int lda, const void* B, int M, int N, int K, const RopeEpi& re,
                      hipStream_t st) {
  if (M == 0) return true;
  if (!gemm_rope_supported(M, N, K)) return false;
  if (gemv_takes(M, N, K, EPI_ROPE) && lda % 8 == 0) {
    launch_gemv_rope(A, lda, B, M, N, K, re, st);
    return true;
  }
  if (ws_prefer(M, N, K, EPI_ROPE) && lda % 8 == 0) {  // 5-16 rows: the weight-streaming MFMA kernel
    launch_ws(A, lda, B, K, nullptr, 0, M, N, K, EPI_ROPE, false, re, 0.f, st);
    return true;
  }
  Plan p = rope_plan(M, N, K);
  if (!((p.BM == 256 || p.variant == 6) && p.BN >= 128)) {  // small M: split-K slabs + fused reduce / RoPE / cache
    float* ws = sk_buf()->ws;
    launch_plan<EPI_NONE, false>(p, (const uint16_t*)A, lda, (const uint16_t*)B, K, nullptr, N, ws,
                                 M, N, K, nullptr, 0, st);
    launch_rope_cache_slabs(re, ws, p.splits, M, N, st);
    return true;
  }
  p.splits = 1;
  p.k_chunk = K;
  launch_plan<EPI_ROPE, false>(p, (const uint16_t*)A, lda, (const uint16_t*)B, K, nullptr, 0, nullptr,
                               M, N, K, nullptr, 0, st, re);
  return true;
}

// The large-M decoder's norm chain: O / down add into the residual and leave per-row sums of
// squares (W4_ADD_SS), gate_up / QKV scale their rows by the RMSNorm factor (W4_RS), so the
// add + RMSNorm passes over [M, H] disappear (norm weights folded into the consumer weights).
// Everything launch_w4_chain needs, so the caller decides the chain ONCE per forward (before the
// first in-place residual update) and never meets a refusal mid-layer: the shape on the
// four-wave kernel, the stream-K scratch that holds the band tickets reserved, and one ticket
// per band of BM rows.
bool w4_chain_ok(int M, int N, int K) {
  if (M <= 0 || gemv_takes(M, N, K, EPI_NONE) || gemv_takes(M, N, K, EPI_ROPE)) return false;
  int cus = 0;
  if (!gemm_sk_available(&cus) || cus <= 0) return false;
  const Plan p = plan(M, N, K, false, 0, 0);
  return (p.variant == 5 || p.variant == 6) && p.splits == 1 && p.BN == 256 && (M + p.BM - 1) / p.BM <= kSkMaxWg &&
         gemm_w4_ok(M, N, K, K, K, N);
}

bool launch_w4_chain(int epi, const void* A, int lda, const void* B, void* C, int ldc, int M, int N, int K,
                     const RopeEpi& re, hipStream_t st) {
  if (M == 0) return true;
  if (!w4_chain_ok(M, N, K) || !gemm_w4_ok(M, N, K, lda, K, ldc)) return false;
  const Plan p = plan(M, N, K, false, 0, 0);
  if (!run_w4(epi, (const uint16_t*)A, lda, (const uint16_t*)B, K, (uint16_t*)C, ldc, M, N, K, st, re, p.BM)) return false;
  return true;
}

// Mid-M norm chain (rows in (decode_chain_max_m, 64], TP = 1): the decoder layer's two add +
// RMSNorm launches (splitk_add_rmsnorm) fold into the planner's small-tile GEMMs.  O / down
// (epi 0) split K and the tile's last split adds into the residual and leaves the row sums of
// squares (mid_chain_finish); gate_up (epi 1, one K range) scales its accumulator rows by the
// RMSNorm factor in its SiLU epilogue; QKV + RoPE (epi 3) takes the factor in the split-K slab
// reduce of the RoPE + cache kernel, or in the weight-streaming kernel's row-scale prologue at
// 5-8 rows (which computes it from the rows it streams).
// gemm_mid_chain op: 0 off (default), 1 on (sc1 hand-off), 2 on (acquire hand-off).  Off by
// default: the in-kernel finish adds ~3.5 us to each O / down call (two ticket round trips,
// write-through partials, the band's row totals) against the ~5 us splitk_add_rmsnorm launch it
// replaces, and the row scale costs gate_up ~0.8 us; interleaved on one box, batch 16 -1 % /
// -3 % and batch 64 -2.6 % / -3.7 % (sc1 / acquire); without the band step (a timing probe,
// numerics off) batch 16 +2-3 % and batch 64 -0.6 % (profiles/r06_mid_chain.md).
static int g_mid_chain = 0;
int gemm_mid_chain(int set) {
  if (set >= 0) g_mid_chain = set;
  return g_mid_chain;
}

bool mid_chain_ok(int M, int N, int K, int epi) {
  if (!g_mid_chain || M <= decode_chain_max_m() || M > 64 || K % kBK || N % 128) return false;
  int cus = 0;
  if (!gemm_sk_available(&cus)) return false;
  if (epi == EPI_ROPE) {
    if (ws_prefer(M, N, K, EPI_ROPE)) return K % 512 == 0;
    const Plan p = rope_plan(M, N, K);
    return !((p.BM == 256 || p.variant == 6) && p.BN >= 128) && rope_slabs_ok(p, M, N);
  }
  const Plan p = plan(M, N, K, false, 0, 0);
  if (p.variant != 0 || p.BM > 64 || N % p.BN) return false;
  if (epi == EPI_SILU_MUL) return p.splits == 1;
  if (epi != EPI_NONE || p.splits < 2) return false;
  const long gx = N / p.BN, gy = (M + p.BM - 1) / p.BM;
  return gx * gy + gy <= kSkMaxWg &&
         (size_t)p.splits * M * N + (size_t)M * gx <= (size_t)2 * kSkMaxWg * 256 * 256;
}

// residual [M, N] += A . B^T in place and ss_tot [M] <- the new rows' sums of squares (epi 0)
bool launch_mid_res_ss(const void* A, int lda, const void* B, void* residual, int ldr, int M, int N, int K,
                       float* ss_tot, hipStream_t st) {
  if (M == 0) return true;
  if (!mid_chain_ok(M, N, K, EPI_NONE)) return false;
  float* ws = nullptr;
  int* cnt = nullptr;
  int cus = 0;
  if (!gemm_sk_scratch(&ws, &cnt, &cus)) return false;
  const Plan p = plan(M, N, K, false, 0, 0);
  RopeEpi re{};
  re.ss_cnt = cnt;
  re.ss_tot = ss_tot;
  re.mid_acq = g_mid_chain == 2;
  launch_plan<EPI_NONE, false>(p, (const uint16_t*)A, lda, (const uint16_t*)B, K, (uint16_t*)residual, ldr, ws, M,
                               N, K, nullptr, 0, st, re);
  return true;
}

// out = SiLU-mul(diag(rsqrt(ss_tot / K + eps)) . A . B^T) (epi 1, gate_up)
bool launch_mid_rs(const void* A, int lda, const void* B, void* out, int ldo, int M, int N, int K,
                   const float* ss_tot, float eps, hipStream_t st) {
  if (M == 0) return true;
  if (!mid_chain_ok(M, N, K, EPI_SILU_MUL)) return false;
  const Plan p = plan(M, N, K, false, 0, 0);
  RopeEpi re{};
  re.ss_in = ss_tot;
  re.ss_inv_k = 1.f / (float)K;
  re.ss_eps = eps;
  launch_plan<EPI_SILU_MUL, false>(p, (const uint16_t*)A, lda, (const uint16_t*)B, K, (uint16_t*)out, ldo, nullptr,
                                   M, N, K, nullptr, 0, st, re);
  return true;
}

long gemm_workspace_floats(int M, int N, int K, int epi) {
  if (gemv_takes(M, N, K, epi)) return 0;
  const Plan p = plan(M, N, K, false, 0, 0);
  return p.splits > 1 ? (long)p.splits * M * N : 0;
}

void launch_gemm(const void* A, int lda, const void* B, int ldb, void* C, int ldc, float* ws,
                 long ws_floats, int M, int N, int K, int epi, hipStream_t st) {
  if (M == 0) return;
  if (gemv_takes(M, N, K, epi) && lda % 8 == 0 && ldb % 8 == 0) {
    launch_gemv(A, lda, B, ldb, C, ldc, M, N, K, epi, st);
    return;
  }
  Plan p = plan(M, N, K, false, 0, 0);
  if (p.splits > 1 && (long)p.splits * M * N > ws_floats) { p.splits = 1; p.k_chunk = K; }
  if (epi == EPI_NONE)
    launch_plan<EPI_NONE, false>(p, (const uint16_t*)A, lda, (const uint16_t*)B, ldb, (uint16_t*)C,
                                 ldc, ws, M, N, K, nullptr, 0, st);
  else
    launch_plan<EPI_SILU_MUL, false>(p, (const uint16_t*)A, lda, (const uint16_t*)B, ldb,
                                     (uint16_t*)C, ldc, ws, M, N, K, nullptr, 0, st);
  if (p.splits > 1) {
    const int outw = epi == EPI_NONE ? N : N / 2;
    const long total = (long)M * (outw / 8);
    const int g = (int)std::min<long>((total + 255) / 256, 4096);
    if (epi == EPI_NONE)
      splitk_reduce_kernel<EPI_NONE><<<g, 256, 0, st>>>((uint16_t*)C, ldc, ws, M, N, p.splits);
    else
      splitk_reduce_kernel<EPI_SILU_MUL><<<g, 256, 0, st>>>((uint16_t*)C, ldc, ws, M, N, p.splits);
  }
}

// y = A.B^T; residual += y; out = rmsnorm(residual) * w.  Returns false (nothing
// launched) when the shape does not take the split-K path: the caller then runs
// gemm + add_rmsnorm.
bool launch_gemm_add_rmsnorm(const void* A, int lda, const void* B, void* out, void* residual,
                             const void* w, float eps, float* ws, long ws_floats, int M, int N,
                             int K, hipStream_t st) {
  if (M == 0) return true;
  if (gemv_takes(M, N, K, EPI_NONE)) return false;  // decode sizes: GEMV + add_rmsnorm (or the norm chain)
  if (ws_prefer(M, N, K, EPI_NONE) && lda % 8 == 0) {
    // 5-16 rows of an O-size projection: the weight-streaming MFMA kernel adds into the residual
    // in place (bf16(res + bf16(y)), norm.hip's rounding), then one RMSNorm pass
    launch_ws(A, lda, B, K, residual, N, M, N, K, 5, false, RopeEpi{}, 0.f, st);
    launch_rmsnorm(out, residual, w, eps, M, N, st);
    return true;
  }
  int splits;
  const Plan p = plan(M, N, K, false, 0, 0);
  if (p.splits <= 1 || p.splits > kMaxSplits || (long)p.splits * M * N > ws_floats || N % 8) return false;
  launch_plan<EPI_NONE, false>(p, (const uint16_t*)A, lda, (const uint16_t*)B, K, nullptr, N, ws,
                               M, N, K, nullptr, 0, st);
  splits = p.splits;
  const int nvec = N / 8;
  int vpt = 1;
  while (vpt < 8 && nvec / vpt > 512) vpt <<= 1;
  const int threads = ((nvec / vpt + 63) / 64) * 64;
  auto* o = (uint16_t*)out;
  auto* r = (uint16_t*)residual;
  auto* wv = (const uint16_t*)w;
  switch (vpt) {
    case 1: splitk_add_rmsnorm_kernel<1><<<M, threads, 0, st>>>(o, r, ws, wv, eps, M, N, splits); break;
    case 2: splitk_add_rmsnorm_kernel<2><<<M, threads, 0, st>>>(o, r, ws, wv, eps, M, N, splits); break;
    case 4: splitk_add_rmsnorm_kernel<4><<<M, threads, 0, st>>>(o, r, ws, wv, eps, M, N, splits); break;
    default: splitk_add_rmsnorm_kernel<8><<<M, threads, 0, st>>>(o, r, ws, wv, eps, M, N, splits); break;
  }
  return true;
}

void launch_grouped_gemm(const void* A, const void* B, void* C, const int* offsets, int n_groups,
                         int M, int N, int K, int max_rows, int epi, hipStream_t st, const int* a_rows,
                         float** defer_ws, int* defer_splits) {
  if (defer_splits) *defer_splits = 1;
  if (M == 0) return;
  if (a_rows == nullptr && defer_splits == nullptr && gemv_grouped_takes(M, N, K, epi)) {  // MoE decode: stream only the routed experts' weights
    launch_gemv_grouped(A, B, C, offsets, n_groups, M, N, K, epi, st);
    return;
  }
  Plan p = plan(M, N, K, true, n_groups, max_rows);
  // Mid-size MoE batches (a few dozen rows per expert): one m-tile per expert x N/64 tiles
  // is too few workgroups to stream every expert's weights at full rate (down at batch 64:
  // 512 workgroups of K = 14336, 4.7 TB/s).  Split K like the dense path, partials in the
  // stream-K slab buffer (same stream, so never in use by another launch), then the reduce
  // kernel applies the epilogue.  Routed tiles are estimated as one m-tile per expert.
  float* ws = nullptr;
  if (p.variant != 3 && K >= 2048 && g_gp[3] != 1 && !(p.nosplit && g_gp[0] <= 0)) {
    const SkBuf* b = sk_buf();
    const long t_est = (long)((N + p.BN - 1) / p.BN) * std::max(1, std::min(n_groups, (M + p.BM - 1) / p.BM + n_groups));
    constexpr int target = 1024;
    int s = (int)std::min<long>(8, std::max<long>(1, target / std::max<long>(1, t_est)));
    if (g_gp[3] > 1) s = g_gp[3];
    while (s > 1 && (K / s) % kBK) --s;
    if (b && s > 1 && (size_t)s * M * N * 4 <= (size_t)2 * kSkMaxWg * 256 * 256 * 4) {
      p.splits = s;
      p.k_chunk = K / s;
      ws = b->ws;
    }
  }
  RopeEpi re{};
  re.a_rows = a_rows;
  if (epi == EPI_NONE)
    launch_plan<EPI_NONE, true>(p, (const uint16_t*)A, K, (const uint16_t*)B, K, (uint16_t*)C, N,
                                ws, M, N, K, offsets, n_groups, st, re);
  else
    launch_plan<EPI_SILU_MUL, true>(p, (const uint16_t*)A, K, (const uint16_t*)B, K, (uint16_t*)C,
                                    N / 2, ws, M, N, K, offsets, n_groups, st, re);
  if (p.splits > 1 && defer_splits != nullptr && epi == EPI_NONE) {  // the caller sums the slabs
    *defer_ws = ws;
    *defer_splits = p.splits;
  } else if (p.splits > 1) {
    const int outw = epi == EPI_NONE ? N : N / 2;
    const long total = (long)M * (outw / 8);
    const int g = (int)std::min<long>((total + 255) / 256, 4096);
    if (epi == EPI_NONE)
      splitk_reduce_kernel<EPI_NONE><<<g, 256, 0, st>>>((uint16_t*)C, N, ws, M, N, p.splits);
    else
      splitk_reduce_kernel<EPI_SILU_MUL><<<g, 256, 0, st>>>((uint16_t*)C, N / 2, ws, M, N, p.splits);
  }
}

}  // namespace mlop
