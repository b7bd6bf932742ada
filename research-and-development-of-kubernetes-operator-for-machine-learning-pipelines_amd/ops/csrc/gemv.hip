// K2: bf16 skinny GEMM / GEMV for decode at M <= 8 rows (default M <= 4: batch-1 .. batch-4 decode).
//
//   C[M, N] = A[M, K] . B[N, K]^T      (A activations, B weights [out, in], both bf16)
//
// At M <= 8 a decode projection is pure weight streaming: every weight byte is read
// once and the arithmetic (M dot products per byte pair) is noise, so the MFMA GEMM's
// LDS ring, 64-row tiles (56+ rows of padding) and split-K slabs are all overhead.
// Here (cdna_hip_programming.md §5 "glds vs register staging", row "GEMV / M <= 16":
// load straight to VGPRs, deep unroll, late vmcnt):
//   * a wave owns 2*RP weight rows; each lane streams 16-B chunks of every row with
//     nontemporal global loads (weights are read by exactly one CU, once:
//     MI355X_MICROARCH.md "nt-weights"), U chunks per row in flight before the
//     first dot: 64 lanes x 16 B = one contiguous 1 KiB run of a row per load
//     instruction;
//   * the activation chunks come through the normal (cached) path: A is a few KiB
//     re-read by every wave from L1/L2;
//   * v_dot2c_f32_bf16 (two bf16 products per op, fp32 accumulate), then a
//     butterfly wave reduction per (row, m) output;
//   * KW = 4 puts the 4 waves of a workgroup on the SAME rows with K interleaved
//     over them (LDS combine) when N alone gives too few waves to keep 256 CUs
//     streaming (70B TP=8 shards: N = 1280 / 1024).
// Epilogues:
//   EPI_NONE      bf16 store;
//   EPI_SILU_MUL  gate/up rows interleaved in groups of 16: a wave takes gate rows
//                 32g+i.. and their up rows 32g+16+i.., so silu(g)*u is formed in
//                 registers and only N/2 columns are stored (gemm.hip's rounding);
//   EPI_ROPE      QKV projection: a wave takes the rotate-half PAIR of rows (d, d+64) of
//                 one q/k head (or two v rows), rotates the bf16-rounded outputs and
//                 stores q to q_out and k / v straight into the paged cache
//                 (rope_cache.hip's math and layouts, no [M, N] round trip, one
//                 launch fewer per layer).
//   EPI_RES       residual (C) += the outputs, in place (the decode norm chain's O / down).
// Prologue RS (the decode norm chain's QKV / gate_up, norm weights folded into B): A is the
// raw residual; each row's sum of squares accumulates from the chunks the dots stream (one
// v_dot2 per chunk, no extra load) and rsqrt(mean + eps) scales the finished sums.
// (Two rejected fusions were removed in round 5: a residual add + RMSNorm prologue that formed A
// from y + residual, and an add + RMSNorm epilogue with a grid ticket.  Both measured slower
// than the decode norm chain above: profiles/r04_decode_small_batch.md.)
#include <stdlib.h>

#include "common.h"
#include "launch.h"

namespace mlop {

namespace {

enum { EPI_NONE = 0, EPI_SILU_MUL = 1, EPI_ROPE = 3, EPI_RES = 5 };
// prologues: none; RS (the row-scale chain: A IS the raw residual and the norm weights are
// folded into B, so the rows' rsqrt(mean(a^2) + eps) comes from the very chunks the dots
// stream: no extra load at all)
enum { PRO_NONE = 0, PRO_RS = 2 };
constexpr int kHeadD = 128;

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;

__device__ __forceinline__ float dot2(uint32_t a, uint32_t b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a), __builtin_bit_cast(bf16x2_t, b),
                                        c, false);
}

__device__ __forceinline__ float dot8(const u32x4& w, const u32x4& x, float c) {
  c = dot2(w.x, x.x, c);
  c = dot2(w.y, x.y, c);
  c = dot2(w.z, x.z, c);
  return dot2(w.w, x.w, c);
}

// acc[r][m] with runtime (r, m) and every index static (the array stays in registers)
template <int R, int M>
__device__ __forceinline__ float acc_pick(const float (&acc)[R][M], int r, int m) {
  float v = 0.f;
#pragma unroll
  for (int rr = 0; rr < R; ++rr)
#pragma unroll
    for (int mm = 0; mm < M; ++mm)
      if (rr == r && mm == m) v = acc[rr][mm];
  return v;
}

// grouped mode (MoE decode, K13 at <= 8 routed rows): rows of A sorted by expert, offsets[E+1]
struct GroupArgs {
  const int* offsets;
  int n_groups;
};

template <int M, int RP, int EPI, int KW, int U, int PRO, bool GROUPED = false>
__global__ void __launch_bounds__(256) gemv_kernel(const uint16_t* __restrict__ A, int lda,
                                                   const uint16_t* __restrict__ B, int ldb,
                                                   uint16_t* __restrict__ C, int ldc, int N, int K,
                                                   RopeEpi re, NormPro np, GroupArgs ga = GroupArgs{}) {
  constexpr int R = 2 * RP;  // weight rows per wave
  constexpr bool RS = PRO == PRO_RS;
  static_assert(EPI != EPI_ROPE || RP == 1, "rope sets are single row pairs");
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // row set: KW == 1 -> one per wave; KW == 4 -> one per workgroup (its waves split K)
  int set = KW == 1 ? blockIdx.x * 4 + wv : blockIdx.x;
  int mc = M;  // rows of A present (grouped: this expert's routed rows)
  if constexpr (GROUPED) {
    // slot = set / (N / R) is the slot-th expert that received rows (the grid covers
    // min(E, M) slots, so experts nobody routed to cost neither a block nor a weight byte)
    const int spg = N / R, slot = set / spg;
    set -= slot * spg;
    int e = -1, seen = 0;
    for (int g = 0; g < ga.n_groups; ++g) {
      if (ga.offsets[g + 1] > ga.offsets[g]) {
        if (seen == slot) { e = g; break; }
        ++seen;
      }
    }
    if (e < 0) return;
    const int m0 = ga.offsets[e];
    mc = min(M, ga.offsets[e + 1] - m0);
    A += (size_t)m0 * lda;
    C += (size_t)m0 * ldc;
    B += (size_t)e * N * ldb;
  } else if (set >= N / R) {
    return;  // every epilogue has N / R sets
  }
  int rows[R];
  if constexpr (EPI == EPI_SILU_MUL) {
    const int col = set * RP, g = col >> 4, i0 = col & 15;  // RP outputs inside one 16-group
#pragma unroll
    for (int p = 0; p < RP; ++p) {
      rows[p] = 32 * g + i0 + p;            // gate
      rows[RP + p] = 32 * g + 16 + i0 + p;  // up
    }
  } else if constexpr (EPI == EPI_ROPE) {
    const int rope_sets = (re.Hq + re.Hkv) * (kHeadD / 2);
    if (set < rope_sets) {
      const int h = set / (kHeadD / 2), d = set % (kHeadD / 2);
      rows[0] = h * kHeadD + d;
      rows[1] = h * kHeadD + kHeadD / 2 + d;
    } else {
      rows[0] = 2 * set;  // v rows: plain consecutive pairs after the q/k rows
      rows[1] = 2 * set + 1;
    }
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r) rows[r] = set * R + r;
  }
  const int KC = K >> 3;  // 16-B chunks per row
  const u32x4* Bv[R];
#pragma unroll
  for (int r = 0; r < R; ++r) Bv[r] = reinterpret_cast<const u32x4*>(B + (size_t)rows[r] * ldb);
  const u32x4* Av[M];
#pragma unroll
  for (int m = 0; m < M; ++m) Av[m] = reinterpret_cast<const u32x4*>(A + (size_t)m * lda);

  float acc[R][M];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int m = 0; m < M; ++m) acc[r][m] = 0.f;
  float ss[M];  // RS: sum of a^2 over this lane's chunks
#pragma unroll
  for (int m = 0; m < M; ++m) ss[m] = 0.f;

  // EPI_ROPE: the epilogue's per-row slot, position and the position's cos / sin are loaded
  // right after the first weight loads are issued, so their round trips (position -> cos / sin
  // is a dependent pair) run under the weight stream instead of after the dot products (lane m
  // holds row m's values; only the waves that store load them)
  const bool rope_lane = EPI == EPI_ROPE && (KW == 1 || wv == 0) && lane < M;
  int pf_slot = -1;
  float pf_c = 0.f, pf_s = 0.f;
  const int rope_d = (set % (kHeadD / 2));
  const bool rope_set = EPI == EPI_ROPE && set < (re.Hq + re.Hkv) * (kHeadD / 2);
  const int lane_off = (KW == 1 ? 0 : wv * 64) + lane;
  // EPI_RES: lane m*R + r adds output (m, set*R + r) into the residual C; its old value is
  // loaded behind the first weight loads (the storing waves only)
  const bool res_lane = EPI == EPI_RES && (KW == 1 || wv == 0) && lane < M * R;
  uint16_t res_pf = 0;
  constexpr int STEP = 64 * KW;  // chunk stride between a lane's consecutive loads
  for (int c0 = 0; c0 < KC; c0 += STEP * U) {
    u32x4 w[U][R], x[U][M];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = c0 + u * STEP + lane_off;
      const bool ok = c < KC;
#pragma unroll
      for (int r = 0; r < R; ++r) w[u][r] = ok ? __builtin_nontemporal_load(Bv[r] + c) : u32x4{0, 0, 0, 0};
#pragma unroll
      for (int m = 0; m < M; ++m) x[u][m] = (ok && m < mc) ? Av[m][c] : u32x4{0, 0, 0, 0};
    }
    if constexpr (EPI == EPI_RES) {
      if (c0 == 0 && res_lane) res_pf = C[(size_t)(lane / R) * ldc + set * R + lane % R];  // behind the weights
    }
    if constexpr (EPI == EPI_ROPE) {
      if (c0 == 0 && rope_lane) {  // issued behind the weight loads
        pf_slot = re.slots[lane];
        if (rope_set) {
          const float* cs = re.cos_sin + (size_t)re.pos[lane] * kHeadD;
          pf_c = cs[rope_d];
          pf_s = cs[kHeadD / 2 + rope_d];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int m = 0; m < M; ++m)
          if (!GROUPED || m < mc) acc[r][m] = dot8(w[u][r], x[u][m], acc[r][m]);  // mc: wave-uniform
      if constexpr (RS) {
#pragma unroll
        for (int m = 0; m < M; ++m) ss[m] = dot8(x[u][m], x[u][m], ss[m]);  // a^2 pairs, fp32 accumulate
      }
    }
  }

#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int m = 0; m < M; ++m) acc[r][m] = wave_sum(acc[r][m]);
  if constexpr (RS) {
#pragma unroll
    for (int m = 0; m < M; ++m) ss[m] = wave_sum(ss[m]);
  }

  if constexpr (KW > 1) {
    constexpr int NV = R * M + (RS ? M : 0);
    __shared__ float red[KW][NV];
    if (lane == 0) {
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int m = 0; m < M; ++m) red[wv][r * M + m] = acc[r][m];
      if constexpr (RS) {
#pragma unroll
        for (int m = 0; m < M; ++m) red[wv][R * M + m] = ss[m];
      }
    }
    __syncthreads();
    if (wv != 0) return;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      float t = 0.f;
#pragma unroll
      for (int k = 0; k < KW; ++k) t += red[k][i];
      if (i < R * M) acc[i / M][i % M] = t;
      else if constexpr (RS) ss[i - R * M] = t;
    }
  }
  if constexpr (RS) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const float inv = rsqrtf(ss[m] / (float)K + np.eps);
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r][m] *= inv;
    }
  }

  // every lane holds every sum now; lane j stores output j of the set
  if constexpr (EPI == EPI_SILU_MUL) {
#pragma unroll
    for (int m = 0; m < M; ++m)
#pragma unroll
      for (int p = 0; p < RP; ++p)
        if (lane == m * RP + p && m < mc)
          C[(size_t)m * ldc + set * RP + p] = f2bf(silu_bf(acc[p][m]) * bf2f(f2bf(acc[RP + p][m])));
  } else if constexpr (EPI == EPI_ROPE) {
    const int rope_sets = (re.Hq + re.Hkv) * (kHeadD / 2);
#pragma unroll
    for (int m = 0; m < M; ++m) {
      if (lane != m) continue;
      const int slot = pf_slot;
      const int blk = slot >= 0 ? slot / re.BS : 0, off = slot >= 0 ? slot % re.BS : 0;
      if (set < rope_sets) {
        const int h = set / (kHeadD / 2), d = set % (kHeadD / 2);
        const float c = pf_c, s = pf_s;
        const float x = bf2f(f2bf(acc[0][m])), y = bf2f(f2bf(acc[1][m]));
        const uint16_t oa = f2bf(x * c - y * s), ob = f2bf(y * c + x * s);
        uint16_t* dst;
        if (h < re.Hq) {
          dst = re.q_out + ((size_t)m * re.Hq + h) * kHeadD;
        } else {
          if (slot < 0) continue;
          dst = re.k_cache + (((size_t)blk * re.Hkv + (h - re.Hq)) * re.BS + off) * kHeadD;
        }
        dst[d] = oa;
        dst[kHeadD / 2 + d] = ob;
      } else if (slot >= 0) {
        const int vr = 2 * set - 2 * rope_sets;  // first v row (0 .. Hkv*128)
        const int kh = vr / kHeadD, dd = vr % kHeadD;
        // token-major page row (as K): dims dd, dd + 1 are adjacent
        uint16_t* dst = re.v_cache + (((size_t)blk * re.Hkv + kh) * re.BS + off) * kHeadD + dd;
        *reinterpret_cast<uint32_t*>(dst) = pack2(acc[0][m], acc[1][m]);
      }
    }
  } else if constexpr (EPI == EPI_RES) {
    // residual (C, in place) = bf16(residual + bf16(y)): norm.hip's add rounding; every element
    // is read and written by its one owning lane only
    if (res_lane) {
      const int m = lane / R, r = lane % R;
      C[(size_t)m * ldc + set * R + r] = f2bf(bf2f(res_pf) + bf2f(f2bf(acc_pick(acc, r, m))));
    }
  } else {
#pragma unroll
    for (int m = 0; m < M; ++m)
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (lane == m * R + r && m < mc) C[(size_t)m * ldc + set * R + r] = f2bf(acc[r][m]);
  }
}

int gemv_max_m() {
  // measured (scripts/history INDEX run38): the GEMV wins every decode projection at M <= 4 in
  // the running model; at M = 8 the 64-row MFMA tiles stream gate_up / down faster
  return 4;
}

// below this many row sets a workgroup's 4 waves share rows and split K (KW = 4): more loads
// in flight per row.  Measured at batch-1/2/4 decode (scripts/run56.sh, run57.sh): at M <= 2
// moving gate_up (7168 sets) to KW = 4 gives +3-4% tok/s at batch 1 and +1.5% at batch 2, at
// M = 4 it loses 5% (the dot work per loaded byte grows with M), and o / qkv / down (2048-3072
// sets) do not move.
int gemv_kw4_sets(int M) { return M <= 2 ? 8192 : 2048; }

template <int M, int EPI, int PRO>
void run_gemv_m(const uint16_t* A, int lda, const uint16_t* B, int ldb, uint16_t* C, int ldc, int N,
                int K, const RopeEpi& re, const NormPro& np, hipStream_t st) {
  constexpr int U = M <= 2 ? 4 : 2;  // chunks per row in flight per lane (VGPR budget)
  // sets of RP row pairs; aim for >= 2048 waves in flight (8 per CU), else KW = 4
  const int pairs = N / 2;
  const int rp = (EPI != EPI_ROPE && pairs / 2 >= 2048) ? 2 : 1;
  const int sets = pairs / rp;
  // the K-split form is for gate_up-size shards, o / down stream as fast without it (run56)
  const bool kw4 = sets < gemv_kw4_sets(M);
#define MLOP_GEMV(RP, KW)                                                                          \
  do {                                                                                             \
    const int blocks = KW == 1 ? cdiv(sets, 4) : sets;                                             \
    gemv_kernel<M, RP, EPI, KW, U, PRO><<<blocks, 256, 0, st>>>(A, lda, B, ldb, C, ldc, N, K, re, \
                                                                  np);                        \
  } while (0)
  if constexpr (EPI == EPI_ROPE) {
    if (kw4) MLOP_GEMV(1, 4); else MLOP_GEMV(1, 1);
  } else {
    if (rp == 2) {
      if (kw4) MLOP_GEMV(2, 4); else MLOP_GEMV(2, 1);
    } else {
      if (kw4) MLOP_GEMV(1, 4); else MLOP_GEMV(1, 1);
    }
  }
#undef MLOP_GEMV
}

template <int EPI, int PRO = PRO_NONE>
void run_gemv(const uint16_t* A, int lda, const uint16_t* B, int ldb, uint16_t* C, int ldc, int M,
              int N, int K, const RopeEpi& re, hipStream_t st, const NormPro& np = NormPro{}) {
  {
    switch (M) {
      case 1: run_gemv_m<1, EPI, PRO>(A, lda, B, ldb, C, ldc, N, K, re, np, st); break;
      case 2: run_gemv_m<2, EPI, PRO>(A, lda, B, ldb, C, ldc, N, K, re, np, st); break;
      case 3: run_gemv_m<3, EPI, PRO>(A, lda, B, ldb, C, ldc, N, K, re, np, st); break;
      case 4: run_gemv_m<4, EPI, PRO>(A, lda, B, ldb, C, ldc, N, K, re, np, st); break;
      case 5: run_gemv_m<5, EPI, PRO>(A, lda, B, ldb, C, ldc, N, K, re, np, st); break;
      case 6: run_gemv_m<6, EPI, PRO>(A, lda, B, ldb, C, ldc, N, K, re, np, st); break;
      case 7: run_gemv_m<7, EPI, PRO>(A, lda, B, ldb, C, ldc, N, K, re, np, st); break;
      default: run_gemv_m<8, EPI, PRO>(A, lda, B, ldb, C, ldc, N, K, re, np, st); break;
    }
  }
}

}  // namespace

// Shapes this path takes: 1 <= M <= MLOP_GEMV_MAX_M (default 4, at most 8), 16-B aligned rows,
// whole row pairs (EPI_NONE), whole 32-row gate/up groups (EPI_SILU_MUL), or a QKV
// projection of 128-wide heads (EPI_ROPE: N = (Hq + 2 Hkv) * 128).
bool gemv_takes(int M, int N, int K, int epi) {
  if (M < 1 || M > gemv_max_m() || K % 8 || N < 4) return false;
  if (epi == EPI_SILU_MUL) return N % 32 == 0;
  if (epi == EPI_ROPE) return N % kHeadD == 0;
  return epi == EPI_NONE && N % 4 == 0;
}

void launch_gemv(const void* A, int lda, const void* B, int ldb, void* C, int ldc, int M, int N, int K,
                 int epi, hipStream_t st) {
  auto* a = (const uint16_t*)A;
  auto* b = (const uint16_t*)B;
  auto* c = (uint16_t*)C;
  const RopeEpi none{};
  if (epi == EPI_SILU_MUL) run_gemv<EPI_SILU_MUL>(a, lda, b, ldb, c, ldc, M, N, K, none, st);
  else run_gemv<EPI_NONE>(a, lda, b, ldb, c, ldc, M, N, K, none, st);
}

void launch_gemv_rope(const void* A, int lda, const void* B, int M, int N, int K, const RopeEpi& re,
                      hipStream_t st) {
  run_gemv<EPI_ROPE>((const uint16_t*)A, lda, (const uint16_t*)B, K, nullptr, 0, M, N, K, re, st);
}

template <int M, int EPI>
void run_gemv_grouped_m(const uint16_t* A, const uint16_t* B, uint16_t* C, int ldc, int N, int K,
                        const int* offsets, int n_groups, hipStream_t st) {
  constexpr int U = M <= 2 ? 4 : 2;
  const int pairs = N / 2;
  const int rp = pairs / 2 >= 2048 ? 2 : 1;
  const int spg = pairs / rp, slots = std::min(n_groups, M);
  const bool kw4 = spg * slots < 2048;
  const GroupArgs ga{offsets, n_groups};
#define MLOP_GEMV_G(RP, KW)                                                                        \
  do {                                                                                             \
    const int sets = spg * slots;                                                                  \
    const int blocks = KW == 1 ? cdiv(sets, 4) : sets;                                             \
    gemv_kernel<M, RP, EPI, KW, U, PRO_NONE, true><<<blocks, 256, 0, st>>>(A, K, B, K, C, ldc, N, K,  \
                                                                          RopeEpi{}, NormPro{}, ga); \
  } while (0)
  if (rp == 2) {
    if (kw4) MLOP_GEMV_G(2, 4); else MLOP_GEMV_G(2, 1);
  } else {
    if (kw4) MLOP_GEMV_G(1, 4); else MLOP_GEMV_G(1, 1);
  }
#undef MLOP_GEMV_G
}

// MoE expert GEMMs at decode: M = routed rows in total (<= 8)
bool gemv_grouped_takes(int M, int N, int K, int epi) {
  return M >= 1 && M <= 8 && K % 8 == 0 && N % (epi == EPI_SILU_MUL ? 32 : 4) == 0 &&
         (epi == EPI_NONE || epi == EPI_SILU_MUL);
}

void launch_gemv_grouped(const void* A, const void* B, void* C, const int* offsets, int n_groups, int M, int N,
                         int K, int epi, hipStream_t st) {
  auto* a = (const uint16_t*)A;
  auto* b = (const uint16_t*)B;
  auto* c = (uint16_t*)C;
  const int ldc = epi == EPI_SILU_MUL ? N / 2 : N;
#define MLOP_GG(MM)                                                                       \
  case MM:                                                                                \
    if (epi == EPI_SILU_MUL) run_gemv_grouped_m<MM, EPI_SILU_MUL>(a, b, c, ldc, N, K, offsets, n_groups, st); \
    else run_gemv_grouped_m<MM, EPI_NONE>(a, b, c, ldc, N, K, offsets, n_groups, st);          \
    break;
  switch (M) {
    MLOP_GG(1) MLOP_GG(2) MLOP_GG(3) MLOP_GG(4) MLOP_GG(5) MLOP_GG(6) MLOP_GG(7) MLOP_GG(8)
    default: break;
  }
#undef MLOP_GG
}

// The decode norm chain (M <= gemv_chain_max_m(), norm weights folded into the consuming projections:
// LlamaModel.fold_norms): O and down add their output into the residual in place (EPI_RES),
// QKV and gate_up read the raw residual and scale each row's sums by rsqrt(mean(a^2) + eps)
// taken from the chunks they stream anyway (PRO_RS).  A decode layer is then five launches
// and no add + RMSNorm pass: the GEMV form of gemm_w4.hip's large-M chain (W4_ADD_SS / W4_RS).
// rows the chain's GEMV form takes (above gemv_max_m() the GEMV takes nothing anyway).
// Measured (scripts/history INDEX r4_chain8): the GEMV with the chain at 6 / 8 rows streams
// 1,419 / 1,612 tok/s against the MFMA path's 1,522 / 1,936 (its split-K reduce already
// carries the add + RMSNorm), so 4 stays.
int gemv_chain_max_m() { return 4; }

bool gemv_chain_takes(int M, int N, int K, int epi) {
  return M <= gemv_chain_max_m() && gemv_takes(M, N, K, epi);
}

void launch_gemv_rs(const void* A, int lda, const void* B, void* C, int ldc, int M, int N, int K, int epi,
                    const RopeEpi& re, float eps, hipStream_t st) {
  auto* a = (const uint16_t*)A;
  auto* b = (const uint16_t*)B;
  auto* c = (uint16_t*)C;
  NormPro np{};
  np.eps = eps;
  if (epi == EPI_SILU_MUL) run_gemv<EPI_SILU_MUL, PRO_RS>(a, lda, b, K, c, ldc, M, N, K, re, st, np);
  else if (epi == EPI_ROPE) run_gemv<EPI_ROPE, PRO_RS>(a, lda, b, K, nullptr, 0, M, N, K, re, st, np);
  else run_gemv<EPI_NONE, PRO_RS>(a, lda, b, K, c, ldc, M, N, K, re, st, np);
}

void launch_gemv_res(const void* A, int lda, const void* B, void* residual, int M, int N, int K, hipStream_t st) {
  run_gemv<EPI_RES>((const uint16_t*)A, lda, (const uint16_t*)B, K, (uint16_t*)residual, N, M, N, K, RopeEpi{}, st);
}

}  // namespace mlop
