// K2 at 5-64 rows (batch 5-64 decode): the weight-streaming MFMA GEMM.
//
//   C[M, N] = A[M, K] . B[N, K]^T      (A activations, B weights [out, in], both bf16)
//
// Between the GEMV (gemv.hip, M <= 4: dot2 on VALU) and the LDS-ring MFMA tiles (gemm.hip),
// a decode projection at 5-64 rows is still pure weight streaming (every weight byte read once,
// ~M / 2 FLOP per byte), but too many dot products for the VALU.  This kernel keeps the GEMV's
// structure -- many waves, each streaming its weight rows straight into registers with
// non-temporal 16-B loads, several K-steps in flight, no LDS ring, no split-K slabs -- and
// does the arithmetic on the matrix cores:
//   * one workgroup = 16 x RB weight rows over the WHOLE K; its 4 waves take one K quarter
//     each (LDS combine at the end), so even O (N = 4096) runs 1024 streaming waves;
//   * a wave's B fragment of one K-step IS the MFMA operand: lane l loads 16 B of weight row
//     (l & 15) at k-chunk (l >> 4) (v_mfma_f32_16x16x32_bf16 B layout, common.h), 16 rows x
//     64 contiguous B per load, the next step continuing the same rows; A fragments come the
//     same way through the cached path (A is a few hundred KiB, L2-resident);
//   * U K-steps in flight per wave (a U-slot register ring: step s's slot is reloaded with
//     step s + U right after its MFMAs), MT = ceil(M / 16) MFMAs per weight fragment.
// Epilogues (the decode norm chain of gemv.hip, so a layer has no add + RMSNorm launch):
//   WS_NONE      bf16 store;
//   WS_RES       residual (C) += y in place, bf16(res + bf16(y)) (norm.hip's add rounding);
//   WS_SILU_MUL  RB = 2: rows 32b.. (gate) and 32b+16.. (up) of the 16-interleaved gate_up;
//   WS_ROPE      RB = 2: a q / k head's rotate-half row pair blocks (d, d + 64), rotated and
//                stored to q_out / the paged K cache; V rows straight into their page rows;
// prologue RS (QKV / gate_up of the chain, norm weights folded into B): A is the raw
// residual; each row's sum of squares accumulates from the very A fragments the MFMAs read
// (4 v_dot2 per fragment) and rsqrt(mean + eps) scales the finished sums.
#include "common.h"
#include "launch.h"

namespace mlop {

namespace {

enum { WS_NONE = 0, WS_SILU_MUL = 1, WS_ROPE = 3, WS_RES = 5 };

typedef __attribute__((ext_vector_type(2))) __bf16 ws_bf16x2;

__device__ __forceinline__ float ws_dot2(uint32_t a, uint32_t b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(ws_bf16x2, a), __builtin_bit_cast(ws_bf16x2, b), c,
                                        false);
}

__device__ __forceinline__ float ws_sq8(const bf16x8& v, float c) {
  const u32x4 w = __builtin_bit_cast(u32x4, v);
  c = ws_dot2(w.x, w.x, c);
  c = ws_dot2(w.y, w.y, c);
  c = ws_dot2(w.z, w.z, c);
  return ws_dot2(w.w, w.w, c);
}

template <int MT, int RB, int U, int EPI, bool RS, bool NT = true>
__global__ void __launch_bounds__(256) gemm_ws_kernel(const uint16_t* __restrict__ A, int lda,
                                                      const uint16_t* __restrict__ B, int ldb,
                                                      uint16_t* __restrict__ C, int ldc, int M, int K,
                                                      RopeEpi re, float eps) {
  static_assert(EPI != WS_SILU_MUL || RB % 2 == 0, "gate / up row block pairs");
  static_assert(EPI != WS_ROPE || RB == 2, "rotate-half row blocks");
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int blk = blockIdx.x;
  constexpr int D = 128;
  // first weight row of each of this workgroup's RB 16-row blocks
  int rbase[RB];
  bool rope_blk = false;
  if constexpr (EPI == WS_SILU_MUL) {  // RB / 2 (gate, up) 16-row group pairs
#pragma unroll
    for (int g = 0; g < RB / 2; ++g) {
      rbase[2 * g] = 32 * (blk * (RB / 2) + g);
      rbase[2 * g + 1] = rbase[2 * g] + 16;
    }
  } else if constexpr (EPI == WS_ROPE) {
    const int rope_blocks = (re.Hq + re.Hkv) * 4;  // 4 blocks of 16 dim pairs per q / k head
    rope_blk = blk < rope_blocks;
    if (rope_blk) {
      rbase[0] = (blk >> 2) * D + (blk & 3) * 16;
      rbase[1] = rbase[0] + D / 2;
    } else {
      rbase[0] = (re.Hq + re.Hkv) * D + (blk - rope_blocks) * 32;
      rbase[1] = rbase[0] + 16;
    }
  } else {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) rbase[rb] = blk * 16 * RB + 16 * rb;
  }

  const int kq = K >> 2;                        // this wave's K quarter
  const int k0 = wv * kq + (lane >> 4) * 8;     // + the lane's 8-element chunk of a 32-k step
  const bf16x8* bp[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
    bp[rb] = reinterpret_cast<const bf16x8*>(B + (size_t)(rbase[rb] + (lane & 15)) * ldb + k0);
  const bf16x8* ap[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t)  // rows past M read row M - 1: their outputs are never stored
    ap[t] = reinterpret_cast<const bf16x8*>(A + (size_t)min(16 * t + (lane & 15), M - 1) * lda + k0);

  f32x4 acc[MT][RB];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) acc[t][rb] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) ss[t] = 0.f;

  // step s = 32 k: element offset 32 s = 4 s bf16x8 vectors
  bf16x8 bq[U][RB], aq[U][MT];
  auto load = [&](int u, int s) {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      if constexpr (NT) bq[u][rb] = __builtin_nontemporal_load(bp[rb] + 4 * s);
      else bq[u][rb] = bp[rb][4 * s];
    }
#pragma unroll
    for (int t = 0; t < MT; ++t) aq[u][t] = ap[t][4 * s];
  };
  auto consume = [&](int u) {
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) acc[t][rb] = mfma16(aq[u][t], bq[u][rb], acc[t][rb]);
    if constexpr (RS) {
#pragma unroll
      for (int t = 0; t < MT; ++t) ss[t] = ws_sq8(aq[u][t], ss[t]);
    }
  };
  // a multiple of U (ws_takes).  The steady-state body reloads unconditionally (a guarded
  // reload made the compiler drain every load, vmcnt(0), at the top of each pass), so each
  // slot's MFMAs wait only for that slot: vmcnt((U - 1) x loads per step)
  const int steps = kq >> 5;
#pragma unroll
  for (int u = 0; u < U; ++u) load(u, u);
  for (int s0 = 0; s0 < steps - U; s0 += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      consume(u);
      load(u, s0 + u + U);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) consume(u);

  // combine the 4 K quarters: red[w][(t RB + rb) 4 + r][lane]; RS: the row sums of squares
  __shared__ float red[4][MT * RB * 4][64];
  __shared__ float red_ss[4][MT][16];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wv][(t * RB + rb) * 4 + r][lane] = acc[t][rb][r];
  if constexpr (RS) {
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const float v = sum_x16_x32(ss[t]);  // lanes l, l^16, l^32, l^48: the four k-chunks of row l & 15
      if (lane < 16) red_ss[wv][t][lane] = v;
    }
  }
  __syncthreads();

  // thread (w', ln) finishes fragment element r = w' of every (t, rb) block: output row
  // m = 16 t + 4 (ln >> 4) + r, weight row rbase[rb] + (ln & 15)
  const int r = wv, ln = lane, col = ln & 15;
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    const int m = 16 * t + 4 * (ln >> 4) + r;
    float y[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const int idx = (t * RB + rb) * 4 + r;
      y[rb] = (red[0][idx][ln] + red[1][idx][ln]) + (red[2][idx][ln] + red[3][idx][ln]);
    }
    if (m >= M) continue;
    if constexpr (RS) {
      const int mr = m & 15;
      const float tot = (red_ss[0][t][mr] + red_ss[1][t][mr]) + (red_ss[2][t][mr] + red_ss[3][t][mr]);
      const float inv = rsqrtf(tot / (float)K + eps);
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) y[rb] *= inv;
    }
    if constexpr (EPI == WS_SILU_MUL) {
#pragma unroll
      for (int g = 0; g < RB / 2; ++g)
        C[(size_t)m * ldc + (blk * (RB / 2) + g) * 16 + col] = f2bf(silu_bf(y[2 * g]) * bf2f(f2bf(y[2 * g + 1])));
    } else if constexpr (EPI == WS_ROPE) {
      const int slot = re.slots[m];
      const int pblk = slot >= 0 ? slot / re.BS : 0, poff = slot >= 0 ? slot % re.BS : 0;
      if (rope_blk) {
        const int h = rbase[0] / D, d = rbase[0] % D + col;  // d < 64
        const float* cs = re.cos_sin + (size_t)re.pos[m] * D;
        const float c = cs[d], s = cs[D / 2 + d];
        const float x = bf2f(f2bf(y[0])), z = bf2f(f2bf(y[1]));
        const uint16_t oa = f2bf(x * c - z * s), ob = f2bf(z * c + x * s);
        uint16_t* dst;
        if (h < re.Hq) {
          dst = re.q_out + ((size_t)m * re.Hq + h) * D;
        } else {
          if (slot < 0) continue;
          dst = re.k_cache + (((size_t)pblk * re.Hkv + (h - re.Hq)) * re.BS + poff) * D;
        }
        dst[d] = oa;
        dst[D / 2 + d] = ob;
      } else if (slot >= 0) {
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
          const int vr = rbase[rb] + col - (re.Hq + re.Hkv) * D;  // v row 0 .. Hkv * 128
          re.v_cache[(((size_t)pblk * re.Hkv + vr / D) * re.BS + poff) * D + vr % D] = f2bf(y[rb]);
        }
      }
    } else if constexpr (EPI == WS_RES) {
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        uint16_t* p = C + (size_t)m * ldc + rbase[rb] + col;
        *p = f2bf(bf2f(*p) + bf2f(f2bf(y[rb])));
      }
    } else {
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) C[(size_t)m * ldc + rbase[rb] + col] = f2bf(y[rb]);
    }
  }
}

// rows the weight-streaming kernel takes, (gemv_chain_max_m, g_ws_max_m]: 0 = off (default, the
// decode chain stays at the GEMV's 4 rows).  Measured slower than the planner's LDS-ring small
// tiles on gate_up / down at every M and on all shapes at M >= 32 (profiles/r06_small_m_ws.md);
// the gemm_ws_max_m op turns it on for A/B runs
int g_ws_max_m = 0;

// A/B plan of the sweep (gemm_ws_plan op, scripts/bench_ws.py): row blocks per workgroup (plain: 1 / 2 /
// 4, SiLU-mul: 2 / 4; 0 = default 1 / 2), K-steps in flight (4 / 8; 0 = 8 where K allows) and
// non-temporal (1) or cached (0, default: 64 B per row per load, the two halves of a line on
// consecutive loads, which the cached path merges in L2 -- 1.3-1.9x faster than nt at o / qkv)
// weight loads.  The RoPE / residual / row-scale forms keep the defaults.
int g_ws_rb = 0, g_ws_u = 0, g_ws_nt = 0;

template <int MT, int RB, int EPI, bool RS, int U, bool NT>
void launch_ws_k(const uint16_t* A, int lda, const uint16_t* B, int ldb, uint16_t* C, int ldc, int M, int N, int K,
                 const RopeEpi& re, float eps, hipStream_t st) {
  gemm_ws_kernel<MT, RB, U, EPI, RS, NT><<<N / (16 * RB), 256, 0, st>>>(A, lda, B, ldb, C, ldc, M, K, re, eps);
}

template <int MT, int RB, int EPI, bool RS>
void run_ws_mt(const uint16_t* A, int lda, const uint16_t* B, int ldb, uint16_t* C, int ldc, int M, int N, int K,
               const RopeEpi& re, float eps, hipStream_t st) {
  const bool u8 = (K >> 2) % (32 * 8) == 0 && g_ws_u != 4;
  constexpr bool SWEEP = !RS && (EPI == WS_NONE || EPI == WS_SILU_MUL);
  if (SWEEP && g_ws_nt) {
    if (u8) launch_ws_k<MT, RB, EPI, RS, 8, true>(A, lda, B, ldb, C, ldc, M, N, K, re, eps, st);
    else launch_ws_k<MT, RB, EPI, RS, 4, true>(A, lda, B, ldb, C, ldc, M, N, K, re, eps, st);
    return;
  }
  if (u8) launch_ws_k<MT, RB, EPI, RS, 8, false>(A, lda, B, ldb, C, ldc, M, N, K, re, eps, st);
  else launch_ws_k<MT, RB, EPI, RS, 4, false>(A, lda, B, ldb, C, ldc, M, N, K, re, eps, st);
}

template <int RB, int EPI, bool RS>
void run_ws(const uint16_t* A, int lda, const uint16_t* B, int ldb, uint16_t* C, int ldc, int M, int N, int K,
            const RopeEpi& re, float eps, hipStream_t st) {
  switch ((M + 15) >> 4) {
    case 1: run_ws_mt<1, RB, EPI, RS>(A, lda, B, ldb, C, ldc, M, N, K, re, eps, st); break;
    case 2: run_ws_mt<2, RB, EPI, RS>(A, lda, B, ldb, C, ldc, M, N, K, re, eps, st); break;
    case 3: run_ws_mt<3, RB, EPI, RS>(A, lda, B, ldb, C, ldc, M, N, K, re, eps, st); break;
    default: run_ws_mt<4, RB, EPI, RS>(A, lda, B, ldb, C, ldc, M, N, K, re, eps, st); break;
  }
}

}  // namespace

int gemm_ws_max_m(int set) {
  if (set >= 0) g_ws_max_m = set > 64 ? 64 : set;
  return g_ws_max_m;
}

// Outside the chain, the plain decode projections take this kernel where it measured faster
// than the planner's small tiles (profiles/r06_small_m_ws.md): the O-size (33 MB) and QKV-size
// (50 MB) matrices at 5-8 rows.  Cold-weight microbench: o 8.4 vs 15.9 us, qkv 12.4 vs 17.8 (the
// QKV form also does RoPE + the paged K/V stores, so the rope_cache slab reduce launch goes);
// in the model the planner's O runs nearer 9 us, so end to end batch 8 gains 1.7 % and batch
// 16 is within noise (-1 %): 8 rows.  gate_up / down and 32+ rows stay on the planner.  The
// gemm_ws_small_m op (0 = off) is the A/B switch.
int g_ws_small_m = 8;

int gemm_ws_small_m(int set) {
  if (set >= 0) g_ws_small_m = set > 64 ? 64 : set;
  return g_ws_small_m;
}

// QKV + RoPE takes the weight-streaming kernel up to g_ws_rope_m rows (gemm_ws_rope_m op): it
// replaces the planner's split-K tile AND the rope_cache slab-reduce launch after it
int g_ws_rope_m = 8;
int gemm_ws_rope_m(int set) {
  if (set >= 0) g_ws_rope_m = set > 64 ? 64 : set;
  return g_ws_rope_m;
}

bool ws_prefer(int M, int N, int K, int epi) {
  if (M <= gemv_chain_max_m() || (long)N * K > 32L * 1024 * 1024 || K % 512) return false;
  if (epi == WS_ROPE) return M <= g_ws_rope_m && N % 128 == 0;
  return M <= g_ws_small_m && (epi == WS_NONE || epi == WS_RES) && N % 16 == 0;
}

void gemm_ws_plan(int rb, int u, int nt) {
  g_ws_rb = rb == 1 || rb == 2 || rb == 4 ? rb : 0;
  g_ws_u = u == 4 || u == 8 ? u : 0;
  g_ws_nt = nt != 0;
}

// Shapes this path takes: gemv_max_m() < M <= ws max (default 64), K a multiple of 512 (four K
// quarters of whole 4-step rings), 16-B aligned rows, whole 16-row blocks (plain / residual),
// whole 32-row gate / up groups (SiLU-mul), a QKV projection of 128-wide heads (RoPE).
bool ws_takes(int M, int N, int K, int epi) {
  if (M <= gemv_chain_max_m() || M > g_ws_max_m || K % 512 || N < 16) return false;
  if (epi == WS_SILU_MUL) return N % 32 == 0;
  if (epi == WS_ROPE) return N % 128 == 0;
  return (epi == WS_NONE || epi == WS_RES) && N % 16 == 0;
}

int decode_chain_max_m() { return g_ws_max_m > gemv_chain_max_m() ? g_ws_max_m : gemv_chain_max_m(); }

bool decode_chain_takes(int M, int N, int K, int epi) {
  return M <= gemv_chain_max_m() ? gemv_chain_takes(M, N, K, epi) : ws_takes(M, N, K, epi);
}

void launch_ws(const void* A, int lda, const void* B, int ldb, void* C, int ldc, int M, int N, int K, int epi,
               bool rs, const RopeEpi& re, float eps, hipStream_t st) {
  auto* a = (const uint16_t*)A;
  auto* b = (const uint16_t*)B;
  auto* c = (uint16_t*)C;
  if (epi == WS_SILU_MUL) {
    if (rs) run_ws<2, WS_SILU_MUL, true>(a, lda, b, ldb, c, ldc, M, N, K, re, eps, st);
    else if (g_ws_rb == 4 && N % 64 == 0) run_ws<4, WS_SILU_MUL, false>(a, lda, b, ldb, c, ldc, M, N, K, re, eps, st);
    else run_ws<2, WS_SILU_MUL, false>(a, lda, b, ldb, c, ldc, M, N, K, re, eps, st);
  } else if (epi == WS_ROPE) {
    if (rs) run_ws<2, WS_ROPE, true>(a, lda, b, ldb, c, ldc, M, N, K, re, eps, st);
    else run_ws<2, WS_ROPE, false>(a, lda, b, ldb, c, ldc, M, N, K, re, eps, st);
  } else if (epi == WS_RES) {
    run_ws<1, WS_RES, false>(a, lda, b, ldb, c, ldc, M, N, K, re, eps, st);
  } else {
    if (rs) run_ws<1, WS_NONE, true>(a, lda, b, ldb, c, ldc, M, N, K, re, eps, st);
    else if (g_ws_rb == 4 && N % 64 == 0) run_ws<4, WS_NONE, false>(a, lda, b, ldb, c, ldc, M, N, K, re, eps, st);
    else if (g_ws_rb == 2 && N % 32 == 0) run_ws<2, WS_NONE, false>(a, lda, b, ldb, c, ldc, M, N, K, re, eps, st);
    else run_ws<1, WS_NONE, false>(a, lda, b, ldb, c, ldc, M, N, K, re, eps, st);
  }
}

}  // namespace mlop
