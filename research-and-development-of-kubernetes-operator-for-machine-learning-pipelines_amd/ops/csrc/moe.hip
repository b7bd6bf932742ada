// Mixture-of-experts routing kernels for gfx950 (K11 route, K12 permute, K14 combine).
// The expert FFN itself is the grouped MFMA GEMM of gemm.hip (K13).
//
// Everything stays on the device and has static shapes (T*k rows reserved, the
// valid count lives in offsets[n_local]), so an MoE layer can be captured in
// a hipGraph: no host sync to size the permuted batch.
//
// Combine is a deterministic gather (out[t] = sum_j w[t,j] * y[inv[t*k+j]],
// fp32 accumulate, one bf16 rounding), not an atomic scatter: bitwise
// reproducible whatever order the permutation assigned rows in
// (cdna_hip_programming.md App. B "Scatter / gather": store-then-sum form).
#include <stdexcept>

#include "common.h"
#include "launch.h"

namespace mlop {

// one thread per token: softmax over E router logits (bf16 in), top-k, renormalise
__global__ void moe_route_kernel(float* __restrict__ topw, int* __restrict__ topi,
                                 const uint16_t* __restrict__ logits, int T, int E, int k) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  const uint16_t* l = logits + (size_t)t * E;
  float v[64];
  float mx = -INFINITY;
  for (int e = 0; e < E; ++e) {
    v[e] = bf2f(l[e]);
    mx = fmaxf(mx, v[e]);
  }
  float s = 0.f;
  for (int e = 0; e < E; ++e) {
    v[e] = __expf(v[e] - mx);
    s += v[e];
  }
  const float inv = 1.f / s;
  float picked = 0.f;
  unsigned long long used = 0ull;
  for (int j = 0; j < k; ++j) {
    int best = 0;
    float bv = -1.f;
    for (int e = 0; e < E; ++e)
      if (!((used >> e) & 1ull) && v[e] > bv) { bv = v[e]; best = e; }
    used |= 1ull << best;
    topi[t * k + j] = best;
    topw[t * k + j] = bv * inv;
    picked += bv * inv;
  }
  const float rn = picked > 0.f ? 1.f / picked : 0.f;
  for (int j = 0; j < k; ++j) topw[t * k + j] *= rn;
}

// counting sort of the T*k routed slots by local expert (one workgroup)
__global__ void __launch_bounds__(1024) moe_sort_kernel(int* __restrict__ offsets,
                                                       int* __restrict__ src,
                                                       int* __restrict__ inv,
                                                       const int* __restrict__ topi, int n_slots,
                                                       int e0, int n_local) {
  __shared__ int cnt[256];
  __shared__ int base[257];
  for (int e = threadIdx.x; e < n_local; e += blockDim.x) cnt[e] = 0;
  __syncthreads();
  for (int s = threadIdx.x; s < n_slots; s += blockDim.x) {
    const int e = topi[s] - e0;
    inv[s] = (e >= 0 && e < n_local) ? atomicAdd(&cnt[e], 1) : -1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int e = 0; e < n_local; ++e) {
      base[e] = acc;
      offsets[e] = acc;
      acc += cnt[e];
    }
    base[n_local] = acc;
    offsets[n_local] = acc;
  }
  __syncthreads();
  for (int s = threadIdx.x; s < n_slots; s += blockDim.x) {
    const int e = topi[s] - e0;
    if (e >= 0 && e < n_local) {
      const int row = base[e] + inv[s];
      inv[s] = row;
      src[row] = s;
    }
  }
}

// xp[r] = x[src[r] / k] for the valid rows (one workgroup per row)
__global__ void __launch_bounds__(256) moe_gather_kernel(uint16_t* __restrict__ xp,
                                                        const uint16_t* __restrict__ x,
                                                        const int* __restrict__ src,
                                                        const int* __restrict__ offsets,
                                                        int n_local, int k, int H) {
  const int r = blockIdx.x;
  if (r >= offsets[n_local]) return;
  const int t = src[r] / k;
  const uint16_t* a = x + (size_t)t * H;
  uint16_t* b = xp + (size_t)r * H;
  for (int c = threadIdx.x * 8; c < H; c += blockDim.x * 8)
    *reinterpret_cast<u32x4*>(b + c) = *reinterpret_cast<const u32x4*>(a + c);
}

// out[t] = sum_j topw[t, j] * y[inv[t*k + j]]   (slots with inv < 0 are not local: skipped)
__global__ void __launch_bounds__(256) moe_combine_kernel(uint16_t* __restrict__ out,
                                                         const uint16_t* __restrict__ y,
                                                         const int* __restrict__ inv,
                                                         const float* __restrict__ topw, int k,
                                                         int H) {
  const int t = blockIdx.x;
  for (int c = threadIdx.x * 8; c < H; c += blockDim.x * 8) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < k; ++j) {
      const int r = inv[t * k + j];
      if (r < 0) continue;
      const float w = topw[t * k + j];
      u32x4 v = *reinterpret_cast<const u32x4*>(y + (size_t)r * H + c);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[2 * q] += w * lo_bf(v[q]);
        acc[2 * q + 1] += w * hi_bf(v[q]);
      }
    }
    u32x4 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = pack2(acc[2 * q], acc[2 * q + 1]);
    *reinterpret_cast<u32x4*>(out + (size_t)t * H + c) = o;
  }
}

// ---------------------------------------------------------------------------
// Optional prologue (MoePro): the post-attention residual add + RMSNorm that produces x, so
// the O projection's output goes straight into the MoE block (one more launch saved).
struct MoePro {
  const uint16_t* y;   // [T, H] O projection output (nullptr: no prologue, x given)
  uint16_t* residual;  // [T, H] in / out
  const uint16_t* w;   // [H] post-attention norm weight
  float eps;
  uint16_t* xn;        // [T, H] normed x (written)
};

// Decode-size MoE dispatch in ONE launch (T <= kSmallT tokens): router GEMV (bf16-rounded
// logits, as the separate router projection stores them), softmax / top-k / renormalise,
// counting sort by local expert and the row gather.  At batch 1-16 each of the four
// separate launches (router GEMV, route, sort, gather) is a ~5 us graph node doing <1 us of
// work (profiles/r02_mixtral_b1.md); one workgroup does all four back to back.
// Wave w computes the logits of experts w, w+8, ...: the expert's router row is loaded once
// (all of a lane's chunks in flight together) while the wave walks the T activation rows.
constexpr int kSmallT = 16, kMaxE = 64, kDispWaves = 8;

template <int CH>  // 16-B chunks per lane per row: H = CH * 512
__global__ void __launch_bounds__(64 * kDispWaves) moe_dispatch_small_kernel(
    float* __restrict__ topw, int* __restrict__ topi, uint16_t* __restrict__ xp, int* __restrict__ offsets,
    int* __restrict__ src, int* __restrict__ inv, const uint16_t* __restrict__ x,
    const uint16_t* __restrict__ wr, int T, int E, int k, int H, int e0, int n_local, MoePro pro) {
  __shared__ float lg[kSmallT][kMaxE];
  __shared__ int s_topi[kSmallT * 8];
  __shared__ int cnt[kMaxE + 1];
  __shared__ int base[kMaxE + 1];
  __shared__ float red[16];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (pro.y != nullptr) {
    // 0. prologue: residual += y; x = rmsnorm(residual) * w (norm.hip's rounding), x -> pro.xn
    for (int t = 0; t < T; ++t) {
      u32x4 r[2];  // H <= 8192: at most two 8-element chunks per thread
      float ss = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int c = (threadIdx.x + i * 64 * kDispWaves) * 8;
        if (c >= H) continue;
        const u32x4 a = *reinterpret_cast<const u32x4*>(pro.y + (size_t)t * H + c);
        const u32x4 b = *reinterpret_cast<const u32x4*>(pro.residual + (size_t)t * H + c);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          r[i][q] = pack2(lo_bf(a[q]) + lo_bf(b[q]), hi_bf(a[q]) + hi_bf(b[q]));
          ss += lo_bf(r[i][q]) * lo_bf(r[i][q]) + hi_bf(r[i][q]) * hi_bf(r[i][q]);
        }
        *reinterpret_cast<u32x4*>(pro.residual + (size_t)t * H + c) = r[i];
      }
      const float rs = rsqrtf(block_sum(ss, red) / (float)H + pro.eps);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int c = (threadIdx.x + i * 64 * kDispWaves) * 8;
        if (c >= H) continue;
        const u32x4 wv8 = *reinterpret_cast<const u32x4*>(pro.w + c);
        u32x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          o[q] = pack2(bf2f(f2bf(lo_bf(r[i][q]) * rs)) * lo_bf(wv8[q]), bf2f(f2bf(hi_bf(r[i][q]) * rs)) * hi_bf(wv8[q]));
        *reinterpret_cast<u32x4*>(pro.xn + (size_t)t * H + c) = o;
      }
    }
    __syncthreads();  // x is read back below by other threads of this workgroup
    x = pro.xn;
  }
  // 1. router logits: lg[t][e] = bf16(x[t] . wr[e])
  for (int e = wv; e < E; e += kDispWaves) {
    const uint16_t* we = wr + (size_t)e * H + lane * 8;
    u32x4 b[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) b[i] = *reinterpret_cast<const u32x4*>(we + i * 512);
    for (int t = 0; t < T; ++t) {
      const uint16_t* xt = x + (size_t)t * H + lane * 8;
      u32x4 a[CH];
#pragma unroll
      for (int i = 0; i < CH; ++i) a[i] = *reinterpret_cast<const u32x4*>(xt + i * 512);
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < CH; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc += lo_bf(a[i][q]) * lo_bf(b[i][q]) + hi_bf(a[i][q]) * hi_bf(b[i][q]);
      acc = wave_sum(acc);
      if (lane == 0) lg[t][e] = bf2f(f2bf(acc));
    }
  }
  for (int e = threadIdx.x; e <= n_local; e += blockDim.x) cnt[e] = 0;
  __syncthreads();
  // 2. softmax -> top-k -> renormalise (moe_route_kernel's math), one thread per token
  if (threadIdx.x < T) {
    const int t = threadIdx.x;
    float mx = -INFINITY;
    for (int e = 0; e < E; ++e) mx = fmaxf(mx, lg[t][e]);
    float sum = 0.f;
    for (int e = 0; e < E; ++e) sum += __expf(lg[t][e] - mx);
    const float rinv = 1.f / sum;
    float picked = 0.f, wsel[8];
    int isel[8];
    unsigned long long used = 0ull;
    for (int j = 0; j < k; ++j) {
      int best = 0;
      float bv = -1.f;
      for (int e = 0; e < E; ++e) {
        const float v = __expf(lg[t][e] - mx);
        if (!((used >> e) & 1ull) && v > bv) { bv = v; best = e; }
      }
      used |= 1ull << best;
      isel[j] = best;
      wsel[j] = bv * rinv;
      picked += bv * rinv;
    }
    const float rn = picked > 0.f ? 1.f / picked : 0.f;
    for (int j = 0; j < k; ++j) {
      topi[t * k + j] = isel[j];
      topw[t * k + j] = wsel[j] * rn;
      s_topi[t * k + j] = isel[j];
    }
  }
  __syncthreads();
  // 3. counting sort of the T*k slots by local expert (moe_sort_kernel), slot order kept
  const int n_slots = T * k;
  if (threadIdx.x == 0) {
    for (int s = 0; s < n_slots; ++s) {
      const int e = s_topi[s] - e0;
      if (e >= 0 && e < n_local) ++cnt[e];
    }
    int acc = 0;
    for (int e = 0; e < n_local; ++e) {
      base[e] = acc;
      offsets[e] = acc;
      acc += cnt[e];
      cnt[e] = 0;
    }
    offsets[n_local] = acc;
    for (int s = 0; s < n_slots; ++s) {
      const int e = s_topi[s] - e0;
      if (e >= 0 && e < n_local) {
        const int row = base[e] + cnt[e]++;
        inv[s] = row;
        src[row] = s;
        s_topi[s] = row;  // reused: slot -> row for the gather below
      } else {
        inv[s] = -1;
        s_topi[s] = -1;
      }
    }
  }
  __syncthreads();
  // 4. gather: xp[row(s)] = x[s / k]
  const int vpr = H / 8;
  for (int i = threadIdx.x; i < n_slots * vpr; i += blockDim.x) {
    const int s = i / vpr, c = (i % vpr) * 8;
    const int row = s_topi[s];
    if (row >= 0)
      *reinterpret_cast<u32x4*>(xp + (size_t)row * H + c) =
          *reinterpret_cast<const u32x4*>(x + (size_t)(s / k) * H + c);
  }
}

bool moe_dispatch_small_takes(int T, int E, int k, int H) {
  return T >= 1 && T <= kSmallT && E <= kMaxE && k <= 8 && (H == 1024 || H == 2048 || H == 4096 || H == 8192);
}

void launch_moe_dispatch_small(float* topw, int* topi, void* xp, int* offsets, int* src, int* inv, const void* x,
                               const void* wr, int T, int E, int k, int H, int e0, int n_local, const void* pro_y,
                               void* pro_res, const void* pro_w, float pro_eps, void* pro_xn, hipStream_t st) {
  const MoePro pro{(const uint16_t*)pro_y, (uint16_t*)pro_res, (const uint16_t*)pro_w, pro_eps, (uint16_t*)pro_xn};
#define MLOP_DISP(CH)                                                                                       \
  moe_dispatch_small_kernel<CH><<<1, 64 * kDispWaves, 0, st>>>(topw, topi, (uint16_t*)xp, offsets, src, inv, \
                                                               (const uint16_t*)x, (const uint16_t*)wr, T, E, k, \
                                                               H, e0, n_local, pro)
  switch (H) {
    case 1024: MLOP_DISP(2); break;
    case 2048: MLOP_DISP(4); break;
    case 4096: MLOP_DISP(8); break;
    default: MLOP_DISP(16); break;
  }
#undef MLOP_DISP
}

// ---------------------------------------------------------------------------
// MoE dispatch for 16 < T <= kMidT tokens (decode batches and prefill chunks) in ONE launch.  At batch 64 the separate
// route is five ~5 us graph nodes per layer (router GEMM + its split-K reduce, top-k, sort,
// gather: profiles/r05_windows.md), each a few us of work at most.  Here:
//   workgroup w (tokens kMidTok w .., moe_mid_tok): the optional add + RMSNorm prologue, router logits
//     (wave e = expert e: the router row loaded once, bf16-rounded as the separate projection
//     stores them), softmax / top-k / renormalise -> topw, topi (written through, sc1);
//   the LAST workgroup (one agent-scope ticket per launch, reset by it: graph-safe; dispatch
//     order and co-residency are not assumed) counts the T*k slots per local expert and writes
//     offsets, inv (slot -> permuted row) and arow (permuted row -> token row).
// There is no gathered copy: the grouped gate_up GEMM reads x rows through arow.  Rows inside
// an expert come in ticket order (LDS atomics), which changes no value: each row's product is
// independent of its position and the combine gathers by inv.
constexpr int kMidT = 16384;
static int g_mid_max_t = kMidT;  // moe_mid_max_tokens op: in-process A/B of the range
// moe_mid_tok op: tokens per workgroup (2, 4 or 8; the router row is loaded once per
// workgroup, token rows two at a time).  Fewer workgroups = fewer router-row reloads and
// fewer agent-scope tickets on the one counter, more sequential prologue tokens per workgroup.
// 0 (default) = by T: 8 from 2,048 tokens, 4 from 512, else 2.  Mixtral batch 1024 windows,
// 2 / 4 / 8: the 3,060-token mixed step 42.3 / 32.3 / 29.3 us, the 1,024-token decode step
// 17.6 / 13.7 / 14.7 us (profiles/r06_moe_spill.md)
static int g_mid_tok = 0;
int moe_mid_tok(int set) {
  if (set == 0 || set == 2 || set == 4 || set == 8) g_mid_tok = set;
  return g_mid_tok;
}
int moe_mid_max_tokens(int set) {
  if (set >= 0) g_mid_max_t = set < kMidT ? set : kMidT;
  return g_mid_max_t;
}

template <int CH, int kMidTok>
__global__ void __launch_bounds__(64 * kDispWaves) moe_dispatch_mid_kernel(
    float* __restrict__ topw, int* __restrict__ topi, int* __restrict__ offsets, int* __restrict__ arow,
    int* __restrict__ inv, const uint16_t* __restrict__ x, const uint16_t* __restrict__ wr, int T, int E, int k,
    int H, int e0, int n_local, MoePro pro, int* __restrict__ ticket) {
  __shared__ float lg[kMidTok][kMaxE];
  __shared__ int cnt[kMaxE + 1];
  __shared__ int base[kMaxE + 1];
  __shared__ float red[16];
  __shared__ int last;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int t0 = blockIdx.x * kMidTok, nt = min(kMidTok, T - t0);
  if (pro.y != nullptr) {
    // prologue for this workgroup's tokens: residual += y; x = rmsnorm(residual) * w
    for (int t = t0; t < t0 + nt; ++t) {
      u32x4 r[2];
      float ss = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int c = (threadIdx.x + i * 64 * kDispWaves) * 8;
        if (c >= H) continue;
        const u32x4 a = *reinterpret_cast<const u32x4*>(pro.y + (size_t)t * H + c);
        const u32x4 b = *reinterpret_cast<const u32x4*>(pro.residual + (size_t)t * H + c);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          r[i][q] = pack2(lo_bf(a[q]) + lo_bf(b[q]), hi_bf(a[q]) + hi_bf(b[q]));
          ss += lo_bf(r[i][q]) * lo_bf(r[i][q]) + hi_bf(r[i][q]) * hi_bf(r[i][q]);
        }
        *reinterpret_cast<u32x4*>(pro.residual + (size_t)t * H + c) = r[i];
      }
      const float rs = rsqrtf(block_sum(ss, red) / (float)H + pro.eps);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int c = (threadIdx.x + i * 64 * kDispWaves) * 8;
        if (c >= H) continue;
        const u32x4 wv8 = *reinterpret_cast<const u32x4*>(pro.w + c);
        u32x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          o[q] = pack2(bf2f(f2bf(lo_bf(r[i][q]) * rs)) * lo_bf(wv8[q]), bf2f(f2bf(hi_bf(r[i][q]) * rs)) * hi_bf(wv8[q]));
        *reinterpret_cast<u32x4*>(pro.xn + (size_t)t * H + c) = o;
      }
    }
    __syncthreads();  // this workgroup's x rows are read back below by other threads
    x = pro.xn;
  }
  // router logits of this workgroup's tokens
  for (int e = wv; e < E; e += kDispWaves) {
    const uint16_t* we = wr + (size_t)e * H + lane * 8;
    u32x4 b[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) b[i] = *reinterpret_cast<const u32x4*>(we + i * 512);
    // token rows two at a time, both rows' chunks in flight together (with the router row's
    // on the first pair: one latency, not three)
#pragma unroll 1
    for (int tp = 0; tp < kMidTok; tp += 2) {
      u32x4 a[2][CH];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < CH; ++i)
          a[t][i] = *reinterpret_cast<const u32x4*>(x + (size_t)(t0 + min(tp + t, nt - 1)) * H + lane * 8 + i * 512);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < CH; ++i)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            acc += lo_bf(a[t][i][q]) * lo_bf(b[i][q]) + hi_bf(a[t][i][q]) * hi_bf(b[i][q]);
        acc = wave_sum(acc);
        if (lane == 0 && tp + t < nt) lg[tp + t][e] = bf2f(f2bf(acc));
      }
    }
  }
  __syncthreads();
  const auto rs_topi = __builtin_amdgcn_make_buffer_rsrc((void*)topi, 0, T * k * 4, 0x00020000);
  if (threadIdx.x < nt) {  // moe_route_kernel's math
    const int t = threadIdx.x;
    float mx = -INFINITY;
    for (int e = 0; e < E; ++e) mx = fmaxf(mx, lg[t][e]);
    float sum = 0.f;
    for (int e = 0; e < E; ++e) sum += __expf(lg[t][e] - mx);
    const float rinv = 1.f / sum;
    float picked = 0.f, wsel[8];
    int isel[8];
    unsigned long long used = 0ull;
    for (int j = 0; j < k; ++j) {
      int best = 0;
      float bv = -1.f;
      for (int e = 0; e < E; ++e) {
        const float v = __expf(lg[t][e] - mx);
        if (!((used >> e) & 1ull) && v > bv) { bv = v; best = e; }
      }
      used |= 1ull << best;
      isel[j] = best;
      wsel[j] = bv * rinv;
      picked += bv * rinv;
    }
    const float rn = picked > 0.f ? 1.f / picked : 0.f;
    for (int j = 0; j < k; ++j) {
      topw[(t0 + t) * k + j] = wsel[j] * rn;
      // written through (sc1) for the sorting workgroup, which may sit on another XCD
      __builtin_amdgcn_raw_buffer_store_b32(isel[j], rs_topi, (uint32_t)(((t0 + t) * k + j) * 4), 0, 16 /* sc1 */);
    }
  }
  // every wave drains its stores, then one lane takes the ticket (the K-half hand-off of
  // gemm_w4.hip: sc1 stores, vmcnt(0), barrier, relaxed agent-scope counter, sc1 loads)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int tk = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = tk == (int)gridDim.x - 1;
    if (last) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
  }
  __syncthreads();
  if (!last) return;
  // counting sort of the T*k slots by local expert
  const int n_slots = T * k;
  for (int e = threadIdx.x; e <= n_local; e += blockDim.x) cnt[e] = 0;
  __syncthreads();
  // the sc1 loads in batches of kSortChunk per thread, all in flight before the first use: one
  // at a time, each load's latency was paid per slot (a 3,060-token mixed step: 12 slots per
  // thread and pass, ~40 of the launch's 52 us)
  constexpr int kSortChunk = 8;
  auto load_chunk = [&](int s0, int (&ev)[kSortChunk]) {
#pragma unroll
    for (int j = 0; j < kSortChunk; ++j) {
      const int s = s0 + j * (int)blockDim.x + (int)threadIdx.x;  // past n_slots: out of range, reads 0
      ev[j] = __builtin_amdgcn_raw_buffer_load_b32(rs_topi, (uint32_t)(s * 4), 0, 16 /* sc1 */) - e0;
    }
  };
  for (int s0 = 0; s0 < n_slots; s0 += kSortChunk * (int)blockDim.x) {
    int ev[kSortChunk];
    load_chunk(s0, ev);
#pragma unroll
    for (int j = 0; j < kSortChunk; ++j) {
      const int s = s0 + j * (int)blockDim.x + (int)threadIdx.x, e = ev[j];
      if (s < n_slots) inv[s] = (e >= 0 && e < n_local) ? atomicAdd(&cnt[e], 1) : -1;  // rank in its expert
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int e = 0; e < n_local; ++e) {
      base[e] = acc;
      offsets[e] = acc;
      acc += cnt[e];
    }
    offsets[n_local] = acc;
  }
  __syncthreads();
  for (int s0 = 0; s0 < n_slots; s0 += kSortChunk * (int)blockDim.x) {
    int ev[kSortChunk], rk[kSortChunk];
    load_chunk(s0, ev);
#pragma unroll
    for (int j = 0; j < kSortChunk; ++j) {  // this thread's own pass-1 stores: plain loads see them
      const int s = s0 + j * (int)blockDim.x + (int)threadIdx.x;
      rk[j] = s < n_slots ? inv[s] : -1;
    }
#pragma unroll
    for (int j = 0; j < kSortChunk; ++j) {
      const int s = s0 + j * (int)blockDim.x + (int)threadIdx.x, e = ev[j];
      if (s < n_slots && e >= 0 && e < n_local) {
        const int row = base[e] + rk[j];
        inv[s] = row;
        arow[row] = s / k;
      }
    }
  }
}

bool moe_dispatch_mid_takes(int T, int E, int k, int H) {
  return T > kSmallT && T <= g_mid_max_t && E <= kMaxE && k <= 8 && (H == 1024 || H == 2048 || H == 4096 || H == 8192);
}

void launch_moe_dispatch_mid(float* topw, int* topi, int* offsets, int* arow, int* inv, const void* x, const void* wr,
                             int T, int E, int k, int H, int e0, int n_local, const void* pro_y, void* pro_res,
                             const void* pro_w, float pro_eps, void* pro_xn, hipStream_t st) {
  float* ws = nullptr;
  int* ticket = nullptr;
  int cus = 0;
  if (!gemm_sk_scratch(&ws, &ticket, &cus)) throw std::runtime_error("moe_dispatch_mid: stream-K scratch not reserved");
  const MoePro pro{(const uint16_t*)pro_y, (uint16_t*)pro_res, (const uint16_t*)pro_w, pro_eps, (uint16_t*)pro_xn};
  const int tok = g_mid_tok ? g_mid_tok : T >= 2048 ? 8 : T >= 512 ? 4 : 2, grid = (T + tok - 1) / tok;
#define MLOP_DISP_T(CH, TOK)                                                                                         \
  moe_dispatch_mid_kernel<CH, TOK><<<grid, 64 * kDispWaves, 0, st>>>(topw, topi, offsets, arow, inv, (const uint16_t*)x, \
                                                                     (const uint16_t*)wr, T, E, k, H, e0, n_local, pro, ticket)
#define MLOP_DISP(CH)                       \
  if (tok == 8) MLOP_DISP_T(CH, 8);         \
  else if (tok == 4) MLOP_DISP_T(CH, 4);    \
  else MLOP_DISP_T(CH, 2);
  switch (H) {
    case 1024: MLOP_DISP(2); break;
    case 2048: MLOP_DISP(4); break;
    case 4096: MLOP_DISP(8); break;
    default: MLOP_DISP(16); break;
  }
#undef MLOP_DISP
#undef MLOP_DISP_T
}

// combine fused with the decoder's residual add + RMSNorm (one workgroup per token row, 8
// elements per thread: at decode sizes every row's reads are in flight at once):
//   m = bf16(sum_j topw[t, j] * y[inv[t*k + j]])   (moe_combine_kernel's rounding)
//   residual[t] = bf16(residual[t] + m);  out[t] = bf16(bf16(residual[t] * rsqrt(mean sq + eps)) * w)
// SLABS: y is not formed; the grouped down GEMM's fp32 split-K slabs ws[s][R][H] are summed
// here (splitk_reduce_kernel's rounding: one bf16 rounding of the sum), one launch fewer
template <bool SLABS>
__global__ void __launch_bounds__(1024) moe_combine_add_rmsnorm_kernel(
    uint16_t* __restrict__ out, uint16_t* __restrict__ residual, const uint16_t* __restrict__ y,
    const int* __restrict__ inv, const float* __restrict__ topw, const uint16_t* __restrict__ w, float eps,
    int k, int H, const float* __restrict__ ws, int splits, int R) {
  __shared__ float scratch[16];
  const int t = blockIdx.x, c = threadIdx.x * 8;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int j = 0; j < k; ++j) {
    const int row = inv[t * k + j];
    if (row < 0) continue;
    const float wt = topw[t * k + j];
    u32x4 v;
    if constexpr (SLABS) {
      float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int sp = 0; sp < splits; ++sp) {
        const float4* p = reinterpret_cast<const float4*>(ws + ((size_t)sp * R + row) * H + c);
        const float4 x0 = p[0], x1 = p[1];
        a[0] += x0.x; a[1] += x0.y; a[2] += x0.z; a[3] += x0.w;
        a[4] += x1.x; a[5] += x1.y; a[6] += x1.z; a[7] += x1.w;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = pack2(a[2 * q], a[2 * q + 1]);
    } else {
      v = *reinterpret_cast<const u32x4*>(y + (size_t)row * H + c);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      acc[2 * q] += wt * lo_bf(v[q]);
      acc[2 * q + 1] += wt * hi_bf(v[q]);
    }
  }
  const u32x4 res = *reinterpret_cast<const u32x4*>(residual + (size_t)t * H + c);
  const u32x4 wv = *reinterpret_cast<const u32x4*>(w + c);
  u32x4 r;
  float ss = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t m = pack2(acc[2 * q], acc[2 * q + 1]);
    r[q] = pack2(lo_bf(m) + lo_bf(res[q]), hi_bf(m) + hi_bf(res[q]));
    ss += lo_bf(r[q]) * lo_bf(r[q]) + hi_bf(r[q]) * hi_bf(r[q]);
  }
  *reinterpret_cast<u32x4*>(residual + (size_t)t * H + c) = r;
  const float rs = rsqrtf(block_sum(ss, scratch) / (float)H + eps);
  u32x4 o;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    o[q] = pack2(bf2f(f2bf(lo_bf(r[q]) * rs)) * lo_bf(wv[q]), bf2f(f2bf(hi_bf(r[q]) * rs)) * hi_bf(wv[q]));
  *reinterpret_cast<u32x4*>(out + (size_t)t * H + c) = o;
}

bool launch_moe_combine_add_rmsnorm(void* out, void* residual, const void* y, const int* inv, const float* topw,
                                    const void* w, float eps, int T, int k, int H, hipStream_t st) {
  if (T == 0) return true;
  if (H % 512 || H > 8192) return false;  // whole 64-thread waves, <= 1024 threads
  moe_combine_add_rmsnorm_kernel<false><<<T, H / 8, 0, st>>>((uint16_t*)out, (uint16_t*)residual, (const uint16_t*)y,
                                                             inv, topw, (const uint16_t*)w, eps, k, H, nullptr, 0, 0);
  return true;
}

// the MoE block's tail in two launches: grouped down GEMM (its split-K partials left in the
// slab buffer) + the combine that sums them, adds into the residual and normalises.  y [R, H]
// is written only when the GEMM does not split.
bool launch_moe_down_combine_add_rmsnorm(void* out, void* residual, void* y, const void* a, const void* w2,
                                         const int* offsets, int n_groups, int R, int H, int I, int max_rows,
                                         const int* inv, const float* topw, const void* norm_w, float eps, int T,
                                         int k, hipStream_t st) {
  if (T == 0) return true;
  if (H % 512 || H > 8192) return false;
  float* ws = nullptr;
  int splits = 1;
  launch_grouped_gemm(a, w2, y, offsets, n_groups, R, H, I, max_rows, 0, st, nullptr, &ws, &splits);
  if (splits > 1)
    moe_combine_add_rmsnorm_kernel<true><<<T, H / 8, 0, st>>>((uint16_t*)out, (uint16_t*)residual, nullptr, inv, topw,
                                                              (const uint16_t*)norm_w, eps, k, H, ws, splits, R);
  else
    moe_combine_add_rmsnorm_kernel<false><<<T, H / 8, 0, st>>>((uint16_t*)out, (uint16_t*)residual, (const uint16_t*)y,
                                                               inv, topw, (const uint16_t*)norm_w, eps, k, H, nullptr, 0, 0);
  return true;
}

void launch_moe_route(float* topw, int* topi, const void* logits, int T, int E, int k,
                      hipStream_t st) {
  if (T == 0) return;
  moe_route_kernel<<<(T + 127) / 128, 128, 0, st>>>(topw, topi, (const uint16_t*)logits, T, E, k);
}

void launch_moe_permute(void* xp, int* offsets, int* src, int* inv, const void* x, const int* topi,
                        int T, int k, int H, int e0, int n_local, hipStream_t st) {
  moe_sort_kernel<<<1, 1024, 0, st>>>(offsets, src, inv, topi, T * k, e0, n_local);
  if (T * k > 0)
    moe_gather_kernel<<<T * k, 256, 0, st>>>((uint16_t*)xp, (const uint16_t*)x, src, offsets,
                                             n_local, k, H);
}

void launch_moe_combine(void* out, const void* y, const int* inv, const float* topw, int T, int k,
                        int H, hipStream_t st) {
  if (T == 0) return;
  moe_combine_kernel<<<T, 256, 0, st>>>((uint16_t*)out, (const uint16_t*)y, inv, topw, k, H);
}

}  // namespace mlop
