// K2': weight-streaming MFMA GEMM for mid-size decode batches (gemv.hip's M <= 4 .. 64 rows).
// OFF by default (MLOP_WSG_MAX_M / gemm_wsg_config): measured and rejected, see g_max_m below.
//
//   C[M, N] = A[M, K] . B[N, K]^T      (A activations, B weights [out, in], both bf16)
//
// Between the GEMV (M <= 4: v_dot2 on VGPR-streamed weights) and the LDS-DMA MFMA tiles
// (gemm.hip, 64-row tiles) a decode projection is still weight streaming: every weight byte
// is read once and the arithmetic is ~15 % of the MFMA rate.  The LDS-DMA ring there keeps
// ~16 KB of weights in flight per workgroup (gate_up at M = 64 streamed 4.7 TB/s,
// profiles/r02_midbatch_decode.md); here weights go STRAIGHT to VGPRs as MFMA B fragments
// (cdna_hip_programming.md §5 "glds vs register staging", row "GEMV / M <= 16": no LDS round
// trip, deep unroll, the compiler's own counted vmcnt):
//   * lane (n = l & 15, g = l >> 4) of a wave loads W[n0 + 16 f + n][k + 32 j + 8 g .. +8]:
//     exactly the v_mfma_f32_16x16x32_bf16 B fragment of k-chunk j (two chunks = one 128-B
//     line per row per 64-K step), nontemporal (read by one CU, once: MI355X_MICROARCH.md
//     "nt-weights");
//   * A fragments (the batch, a few hundred KB, L2-resident and re-read by every workgroup)
//     come through the cached path into the same register ring;
//   * the 4 waves of a workgroup own the SAME 16 NF columns and interleave the 64-K steps of
//     the workgroup's K range (wave w: steps w, w + 4, ...), so N / (16 NF) workgroups cover
//     the matrix without split-K slabs; their partial tiles are summed through LDS once;
//   * U steps of both operands in flight per wave (U x 2 (NF + MT) x 16 B per lane), 2 waves
//     per SIMD: 100+ KB of weights in flight per CU;
//   * narrow N (o / down / qkv at 16-32 columns per workgroup give < 256 workgroups): K is
//     split over workgroups into fp32 slabs [s][M][N]; gemm.hip's reduce kernels apply the
//     epilogue (SiLU-mul) or the decoder's residual add + RMSNorm.  ws != nullptr selects the
//     slab store (also with one split: the fused add + RMSNorm reads the fp32 tile).
// Epilogues without slabs: EPI_NONE bf16; EPI_SILU_MUL (gate / up rows interleaved in groups
// of 16, gemm.hip's rounding) stores N/2 columns.
#include <stdlib.h>

#include "common.h"
#include "launch.h"

namespace mlop {

namespace {

enum { EPI_NONE = 0, EPI_SILU_MUL = 1 };
constexpr int kKS = 64;  // K per step: two MFMA k-chunks

template <int MT, int NF, int U>
__global__ void __launch_bounds__(256, 2) wsg_kernel(const uint16_t* __restrict__ A, int lda,
                                                     const uint16_t* __restrict__ B, int ldb,
                                                     uint16_t* __restrict__ C, int ldc,
                                                     float* __restrict__ ws, int M, int N, int K,
                                                     int k_chunk, int nblk, int epi) {
  constexpr int CW = 16 * NF, RW = 16 * MT, LDR = CW + 4;
  __shared__ __attribute__((aligned(16))) float red[4 * RW * LDR];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nb = blockIdx.x % nblk, s = blockIdx.x / nblk;
  const int n0 = nb * CW;
  const int kbeg = s * k_chunk;
  const int kend = min(K, kbeg + k_chunk);
  const int nsteps = (kend - kbeg) / kKS;
  const int my = nsteps > w ? (nsteps - w + 3) / 4 : 0;  // this wave's steps: w, w + 4, ...
  const int r16 = lane & 15, g = lane >> 4;

  const bf16x8* bp[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f)
    bp[f] = reinterpret_cast<const bf16x8*>(B + (size_t)(n0 + 16 * f + r16) * ldb + kbeg + w * kKS + 8 * g);
  const bf16x8* ap[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t)
    ap[t] = reinterpret_cast<const bf16x8*>(A + (size_t)min(16 * t + r16, M - 1) * lda + kbeg + w * kKS + 8 * g);
  constexpr int STEP = 4 * kKS / 8;  // bf16x8 units between a wave's steps

  bf16x8 bq[U][NF][2], aq[U][MT][2];
  auto load = [&](int slot, int t) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
#pragma unroll
      for (int f = 0; f < NF; ++f) bq[slot][f][j] = __builtin_nontemporal_load(bp[f] + t * STEP + 4 * j);
#pragma unroll
      for (int m = 0; m < MT; ++m) aq[slot][m][j] = ap[m][t * STEP + 4 * j];
    }
  };

  f32x4 acc[MT][NF];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int f = 0; f < NF; ++f) acc[m][f] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int slot) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int f = 0; f < NF; ++f)
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m][f] = mfma16(aq[slot][m][j], bq[slot][f][j], acc[m][f]);
  };
  // Steady state without a data-dependent branch around any load: the compiler's vmcnt
  // accounting merges the states of both sides of such a branch and then waits as if the
  // prefetches had not been issued (drains the ring to one step).  Step t lives in slot t % U.
  int t0 = 0;
  if (my >= 2 * U - 1) {
#pragma unroll
    for (int u = 0; u < U - 1; ++u) {
      load(u, u);  // in slot order: the loop's vmcnt counts assume it
      __builtin_amdgcn_sched_barrier(0);
    }
    for (; t0 + 2 * U - 2 < my; t0 += U) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        // sched_barrier: keep the prefetch ahead of the MFMAs (the scheduler otherwise sinks
        // each load next to its use and the ring degenerates to load-then-wait)
        load((u + U - 1) % U, t0 + u + U - 1);
        __builtin_amdgcn_sched_barrier(0);
        compute(u);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  } else {
#pragma unroll
    for (int u = 0; u < U - 1; ++u)
      if (u < my) load(u, u);
  }
  // tail (< 2U - 1 steps; t0 is a multiple of U, steps t0 .. t0 + U - 2 already in flight)
#pragma unroll
  for (int u = 0; u < 2 * U - 1; ++u) {
    const int t = t0 + u;
    if (t < my) {
      if (t + U - 1 < my) load((u + U - 1) % U, t + U - 1);
      compute(u % U);
    }
  }

  // the 4 waves' partial tiles -> LDS, summed by all 256 threads
  float* mine = red + w * RW * LDR;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
      for (int i = 0; i < 4; ++i) mine[(16 * m + 4 * g + i) * LDR + 16 * f + r16] = acc[m][f][i];
  __syncthreads();
  auto sum8 = [&](int r, int c, float* o) {
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4* p = reinterpret_cast<const float4*>(red + (q * RW + r) * LDR + c);
      const float4 x = p[0], y = p[1];
      o[0] += x.x; o[1] += x.y; o[2] += x.z; o[3] += x.w;
      o[4] += y.x; o[5] += y.y; o[6] += y.z; o[7] += y.w;
    }
  };
  const int rows = min(RW, M);
  if (ws != nullptr) {  // fp32 slab [s][M][N]; gemm.hip's reduce applies the epilogue
    constexpr int VPR = CW / 8;
    for (int v = threadIdx.x; v < RW * VPR; v += 256) {
      const int r = v / VPR, c = (v % VPR) * 8;
      if (r >= rows) continue;
      float o[8];
      sum8(r, c, o);
      float4* d = reinterpret_cast<float4*>(ws + ((size_t)s * M + r) * N + n0 + c);
      d[0] = float4{o[0], o[1], o[2], o[3]};
      d[1] = float4{o[4], o[5], o[6], o[7]};
    }
  } else if (epi == EPI_NONE) {
    constexpr int VPR = CW / 8;
    for (int v = threadIdx.x; v < RW * VPR; v += 256) {
      const int r = v / VPR, c = (v % VPR) * 8;
      if (r >= rows) continue;
      float o[8];
      sum8(r, c, o);
      u32x4 out;
#pragma unroll
      for (int j = 0; j < 4; ++j) out[j] = pack2(o[2 * j], o[2 * j + 1]);
      *reinterpret_cast<u32x4*>(C + (size_t)r * ldc + n0 + c) = out;
    }
  } else {  // EPI_SILU_MUL: columns 32q .. 32q+15 gate, 32q+16 .. 32q+31 up (NF even)
    constexpr int VPR = CW / 16;
    for (int v = threadIdx.x; v < RW * VPR; v += 256) {
      const int r = v / VPR, j0 = (v % VPR) * 8;
      if (r >= rows) continue;
      const int gc = (j0 / 16) * 32 + (j0 % 16);
      float gt[8], up[8];
      sum8(r, gc, gt);
      sum8(r, gc + 16, up);
      u32x4 out;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        out[j] = pack2(silu_bf(gt[2 * j]) * bf2f(f2bf(up[2 * j])), silu_bf(gt[2 * j + 1]) * bf2f(f2bf(up[2 * j + 1])));
      *reinterpret_cast<u32x4*>(C + (size_t)r * ldc + n0 / 2 + j0) = out;
    }
  }
}

int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

// rows handled here and the workgroup count below which K is split into slabs; both settable at
// run time for in-process A/B.  Default 0 = OFF: measured slower than gemm.hip's LDS-DMA tiles
// (profiles/r02_wsgemm_rejected.md): a B fragment loaded straight from memory is a 16-row x 64-B
// access shape, which streams at 4.4 TB/s where 8-row x 128-B pieces reach 5.5 (scripts/bw_shapes.hip)
int g_max_m = env_int("MLOP_WSG_MAX_M", 0);
int g_min_wg = env_int("MLOP_WSG_MIN_WG", 256);

int pick_nf(int mt, int N) {
  if (mt >= 4) return 2;
  return (N % 64 == 0 && N / 64 >= g_min_wg) ? 4 : 2;
}

}  // namespace

int wsg_config(int max_m, int min_wg) {
  if (max_m >= 0) g_max_m = max_m;
  if (min_wg >= 0) g_min_wg = min_wg;
  return g_max_m;
}

bool wsg_takes(int M, int N, int K, int epi) {
  if (M < 1 || M > g_max_m || M > 64 || K % kKS || (epi != EPI_NONE && epi != EPI_SILU_MUL)) return false;
  const int mt = (M + 15) / 16;
  return N % (16 * pick_nf(mt == 3 ? 4 : mt, N)) == 0 && (epi == EPI_NONE || N % 32 == 0);
}

// K splits (1 = none) for this shape: enough workgroups for one per CU (g_min_wg)
int wsg_splits(int M, int N, int K, int epi) {
  (void)epi;
  int mt = (M + 15) / 16;
  if (mt == 3) mt = 4;
  const int nblk = N / (16 * pick_nf(mt, N));
  int s = nblk >= g_min_wg ? 1 : std::min(8, (g_min_wg + nblk - 1) / nblk);
  const int steps = K / kKS;
  s = std::max(1, std::min(s, steps / 4));  // >= 4 steps (one per wave) per split
  const int spl = (steps + s - 1) / s;
  return (steps + spl - 1) / spl;
}

// ws: fp32 slabs [splits][M][N] (any splits >= 1) or nullptr (epilogue store, splits == 1).
// Returns the number of slabs written (<= splits).
int launch_wsg(const void* Av, int lda, const void* Bv, int ldb, void* Cv, int ldc, float* ws, int M, int N,
                int K, int epi, int splits, hipStream_t st) {
  auto* A = (const uint16_t*)Av;
  auto* B = (const uint16_t*)Bv;
  auto* C = (uint16_t*)Cv;
  int mt = (M + 15) / 16;
  if (mt == 3) mt = 4;
  const int nf = pick_nf(mt, N);
  const int nblk = N / (16 * nf);
  const int steps = K / kKS;
  const int spl = (steps + splits - 1) / splits;  // steps per split
  const int k_chunk = spl * kKS;
  const int grid = nblk * ((steps + spl - 1) / spl);
#define MLOP_WSG(MT_, NF_, U_) \
  wsg_kernel<MT_, NF_, U_><<<grid, 256, 0, st>>>(A, lda, B, ldb, C, ldc, ws, M, N, K, k_chunk, nblk, epi)
  if (mt == 1) {
    if (nf == 4) MLOP_WSG(1, 4, 4); else MLOP_WSG(1, 2, 4);
  } else if (mt == 2) {
    if (nf == 4) MLOP_WSG(2, 4, 3); else MLOP_WSG(2, 2, 4);
  } else {
    MLOP_WSG(4, 2, 3);
  }
#undef MLOP_WSG
  return grid / nblk;
}

}  // namespace mlop
