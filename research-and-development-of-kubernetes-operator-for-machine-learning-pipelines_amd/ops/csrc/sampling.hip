// Token sampling (K10) for gfx950: greedy argmax and temperature/top-k/top-p.
//
// One workgroup (256 threads = 4 waves) per logits row ([n, V] fp32, V up to
// ~256k).  Top-k WITHOUT a full-vocab sort: an exact 4-pass 8-bit radix select
// finds the K-th largest key (monotone uint image of the float), the >= K
// candidates are gathered into LDS, bitonic-sorted (K <= 1024), and the draw
// is an inverse-CDF walk over the block-wide prefix sum of exp((l - l_max)/T),
// truncated at the top-p mass.  Rows re-read in each pass come from L2/MALL
// (a 128k-vocab row is 512 KB), the kernel is a few tens of microseconds for
// a 256-row decode batch.
#include <algorithm>

#include "common.h"
#include "launch.h"

namespace mlop {

constexpr int kSampleThreads = 256;
constexpr int kMaxCand = 1024;

__device__ __forceinline__ uint32_t fkey(float f) {
  uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

// (value, index) argmax with ties to the smallest index; NaN never wins
__device__ __forceinline__ void amax_merge(float& v, int& i, float ov, int oi) {
  if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
}

__device__ void block_argmax(const float* __restrict__ row, int V, float* sv, int* si,
                             float& best_v, int& best_i) {
  float v = -INFINITY;
  int idx = 0x7fffffff;
  const int nv4 = V >> 2;
  const float4* r4 = reinterpret_cast<const float4*>(row);
  for (int j = threadIdx.x; j < nv4; j += blockDim.x) {
    float4 x = r4[j];
    amax_merge(v, idx, x.x, 4 * j);
    amax_merge(v, idx, x.y, 4 * j + 1);
    amax_merge(v, idx, x.z, 4 * j + 2);
    amax_merge(v, idx, x.w, 4 * j + 3);
  }
  for (int j = (nv4 << 2) + threadIdx.x; j < V; j += blockDim.x) amax_merge(v, idx, row[j], j);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float ov = __shfl_xor(v, o, 64);
    int oi = __shfl_xor(idx, o, 64);
    amax_merge(v, idx, ov, oi);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sv[wid] = v; si[wid] = idx; }
  __syncthreads();
  best_v = sv[0];
  best_i = si[0];
  for (int w = 1; w < (int)(blockDim.x >> 6); ++w) amax_merge(best_v, best_i, sv[w], si[w]);
  __syncthreads();
}

__global__ void __launch_bounds__(kSampleThreads) argmax_kernel(long* __restrict__ out,
                                                               const float* __restrict__ logits,
                                                               int V, long ld) {
  __shared__ float sv[kSampleThreads / 64];
  __shared__ int si[kSampleThreads / 64];
  float bv;
  int bi;
  block_argmax(logits + blockIdx.x * ld, V, sv, si, bv, bi);
  if (threadIdx.x == 0) out[blockIdx.x] = bi == 0x7fffffff ? 0 : bi;
}

// greedy over bf16 logits straight from the LM-head GEMM (no fp32 copy of the
// [n, V] logits): 8 values per 16-B load; bf16 -> f32 is exact, so ties and the
// result equal the fp32 path's
__global__ void __launch_bounds__(kSampleThreads) argmax_bf16_kernel(long* __restrict__ out,
                                                                    const uint16_t* __restrict__ logits,
                                                                    int V, long ld) {
  __shared__ float sv[kSampleThreads / 64];
  __shared__ int si[kSampleThreads / 64];
  const uint16_t* row = logits + blockIdx.x * ld;
  float v = -INFINITY;
  int idx = 0x7fffffff;
  const int nv8 = V >> 3;
  const u32x4* r8 = reinterpret_cast<const u32x4*>(row);
  for (int j = threadIdx.x; j < nv8; j += blockDim.x) {
    const u32x4 x = r8[j];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      amax_merge(v, idx, lo_bf(x[k]), 8 * j + 2 * k);
      amax_merge(v, idx, hi_bf(x[k]), 8 * j + 2 * k + 1);
    }
  }
  for (int j = (nv8 << 3) + threadIdx.x; j < V; j += blockDim.x) amax_merge(v, idx, bf2f(row[j]), j);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float ov = __shfl_xor(v, o, 64);
    int oi = __shfl_xor(idx, o, 64);
    amax_merge(v, idx, ov, oi);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sv[wid] = v; si[wid] = idx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float bv = sv[0];
    int bi = si[0];
    for (int w = 1; w < kSampleThreads / 64; ++w) amax_merge(bv, bi, sv[w], si[w]);
    out[blockIdx.x] = bi == 0x7fffffff ? 0 : bi;
  }
}

// Small decode batches (n rows << 256 CUs): one workgroup per row streams a 256 KB row
// at a single CU's rate (~46 us for 128k vocab).  Split each row over S workgroups; each
// writes its (value, index) as one ordered 64-bit key (max key = max value, ties to the
// smallest index), and a one-wave-per-row pass picks the max of the S keys.
__device__ __forceinline__ unsigned long long amax_key(float v, int i) {
  return ((unsigned long long)fkey(v) << 32) | (unsigned long long)(0xffffffffu - (uint32_t)i);
}

__global__ void __launch_bounds__(kSampleThreads) argmax_bf16_split_kernel(
    unsigned long long* __restrict__ keys, const uint16_t* __restrict__ logits, int V, long ld, int S) {
  __shared__ float sv[kSampleThreads / 64];
  __shared__ int si[kSampleThreads / 64];
  const int s = blockIdx.x, row_id = blockIdx.y;
  const uint16_t* row = logits + row_id * ld;
  const int nv8 = V >> 3, per = (nv8 + S - 1) / S;
  const int j0 = s * per, j1 = min(nv8, j0 + per);
  float v = -INFINITY;
  int idx = 0x7fffffff;
  const u32x4* r8 = reinterpret_cast<const u32x4*>(row);
  for (int j = j0 + threadIdx.x; j < j1; j += blockDim.x) {
    const u32x4 x = r8[j];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      amax_merge(v, idx, lo_bf(x[k]), 8 * j + 2 * k);
      amax_merge(v, idx, hi_bf(x[k]), 8 * j + 2 * k + 1);
    }
  }
  if (s == S - 1)
    for (int j = (nv8 << 3) + threadIdx.x; j < V; j += blockDim.x) amax_merge(v, idx, bf2f(row[j]), j);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float ov = __shfl_xor(v, o, 64);
    int oi = __shfl_xor(idx, o, 64);
    amax_merge(v, idx, ov, oi);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sv[wid] = v; si[wid] = idx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float bv = sv[0];
    int bi = si[0];
    for (int w = 1; w < kSampleThreads / 64; ++w) amax_merge(bv, bi, sv[w], si[w]);
    keys[(size_t)row_id * S + s] = amax_key(bv, bi);
  }
}

__global__ void __launch_bounds__(64) argmax_keys_kernel(long* __restrict__ out,
                                                         const unsigned long long* __restrict__ keys,
                                                         int S) {
  const int row_id = blockIdx.x, lane = threadIdx.x;
  unsigned long long k = 0;
  for (int s = lane; s < S; s += 64) k = max(k, keys[(size_t)row_id * S + s]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t hi = __shfl_xor((uint32_t)(k >> 32), o, 64), lo = __shfl_xor((uint32_t)k, o, 64);
    k = max(k, ((unsigned long long)hi << 32) | lo);
  }
  if (lane == 0) {
    const int i = (int)(0xffffffffu - (uint32_t)k);
    out[row_id] = (k == 0 || i == 0x7fffffff) ? 0 : i;
  }
}

// idx_map (optional): the row holds pre-selected candidates (sample_presel_kernel) and
// idx_map[row * ld + j] is candidate j's vocabulary index (-inf padding maps to 0x7fffffff)
__global__ void __launch_bounds__(kSampleThreads) sample_kernel(
    long* __restrict__ out, const float* __restrict__ logits, int V, long ld,
    const float* __restrict__ temps, const int* __restrict__ top_ks,
    const float* __restrict__ top_ps, const float* __restrict__ uniform,
    const int* __restrict__ idx_map = nullptr) {
  __shared__ uint32_t hist[256];
  __shared__ float cv[kMaxCand];
  __shared__ int ci[kMaxCand];
  __shared__ float scan[kMaxCand];
  __shared__ float sv[kSampleThreads / 64];
  __shared__ int si[kSampleThreads / 64];
  __shared__ uint32_t s_prefix, s_remaining, s_cnt_gt, s_cnt_eq;

  const int row_id = blockIdx.x;
  const float* row = logits + row_id * ld;
  const float T = temps[row_id];
  if (T <= 0.f) {
    float bv;
    int bi;
    block_argmax(row, V, sv, si, bv, bi);
    if (idx_map && bi != 0x7fffffff) bi = idx_map[row_id * ld + bi];
    if (threadIdx.x == 0) out[row_id] = bi == 0x7fffffff ? 0 : bi;
    return;
  }
  int K = top_ks[row_id];
  if (K <= 0 || K > kMaxCand) return;  // full-vocabulary rows: sample_full_kernel
  if (K > V) K = V;

  // ---- exact radix select of the K-th largest key (4 x 8-bit digits, MSB first)
  uint32_t prefix = 0, mask = 0, remaining = (uint32_t)K;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int b = threadIdx.x; b < 256; b += blockDim.x) hist[b] = 0;
    __syncthreads();
    for (int j = threadIdx.x; j < V; j += blockDim.x) {
      const uint32_t k = fkey(row[j]);
      if ((k & mask) == prefix) atomicAdd(&hist[(k >> shift) & 0xff], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t above = 0;
      int d = 255;
      for (; d > 0; --d) {
        if (above + hist[d] >= remaining) break;
        above += hist[d];
      }
      s_prefix = prefix | ((uint32_t)d << shift);
      s_remaining = remaining - above;
    }
    __syncthreads();
    prefix = s_prefix;
    remaining = s_remaining;
    mask |= 0xffu << shift;
  }
  // keys > prefix: K - remaining of them; keys == prefix: take `remaining`
  if (threadIdx.x == 0) { s_cnt_gt = 0; s_cnt_eq = 0; }
  __syncthreads();
  const uint32_t n_gt = (uint32_t)K - remaining;
  for (int j = threadIdx.x; j < V; j += blockDim.x) {
    const float x = row[j];
    const uint32_t k = fkey(x);
    if (k > prefix) {
      const uint32_t p = atomicAdd(&s_cnt_gt, 1u);
      if (p < n_gt) { cv[p] = x; ci[p] = idx_map ? idx_map[row_id * ld + j] : j; }
    } else if (k == prefix) {
      const uint32_t p = atomicAdd(&s_cnt_eq, 1u);
      if (p < remaining) { cv[n_gt + p] = x; ci[n_gt + p] = idx_map ? idx_map[row_id * ld + j] : j; }
    }
  }
  __syncthreads();
  // pad to a power of two for the bitonic network
  int P = 1;
  while (P < K) P <<= 1;
  for (int j = K + threadIdx.x; j < P; j += blockDim.x) { cv[j] = -INFINITY; ci[j] = 0x7fffffff; }
  __syncthreads();
  // ---- bitonic sort, descending by value, ties by ascending index
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < P / 2; t += blockDim.x) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool desc = ((lo & size) == 0);
        const float a = cv[lo], b = cv[hi];
        const int ia = ci[lo], ib = ci[hi];
        const bool a_first = (a > b) || (a == b && ia < ib);
        if (a_first != desc) {
          cv[lo] = b; cv[hi] = a;
          ci[lo] = ib; ci[hi] = ia;
        }
      }
      __syncthreads();
    }
  }
  // ---- softmax over candidates + inclusive prefix sum (Hillis-Steele in LDS)
  const float vmax = cv[0];
  const float invT = 1.f / T;
  for (int j = threadIdx.x; j < P; j += blockDim.x)
    scan[j] = j < K ? __expf((cv[j] - vmax) * invT) : 0.f;
  __syncthreads();
  for (int o = 1; o < P; o <<= 1) {
    float add[kMaxCand / kSampleThreads];
    int c = 0;
    for (int j = threadIdx.x; j < P; j += blockDim.x, ++c) add[c] = j >= o ? scan[j - o] : 0.f;
    __syncthreads();
    c = 0;
    for (int j = threadIdx.x; j < P; j += blockDim.x, ++c) scan[j] += add[c];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float total = scan[K - 1];
    const float p = top_ps[row_id];
    int cut = K - 1;
    if (p < 1.f) {
      const float lim = p * total;
      int lo = 0, hi = K - 1;  // first index with scan >= lim
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (scan[mid] >= lim) hi = mid; else lo = mid + 1;
      }
      cut = lo;
    }
    const float target = uniform[row_id] * scan[cut];
    int lo = 0, hi = cut;  // first index with scan > target
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (scan[mid] > target) hi = mid; else lo = mid + 1;
    }
    out[row_id] = ci[lo] == 0x7fffffff ? 0 : ci[lo];
  }
}

// Small batches: one workgroup per row makes sample_kernel a ~0.5 ms single-CU job over a
// 128k vocabulary (5 dependent passes over 512 KB).  Stage 1 splits each row over S
// workgroups: a workgroup stages its slice (<= kPreselSlice floats) in LDS once, radix-
// selects the slice's own top-K (K = the row's top_k, capped at kMaxCand) and writes them as
// kMaxCand (value, vocab index) candidates (-inf padding).  The row's global top-K is inside
// the union of the slices' top-K, so stage 2 (sample_kernel over the S * kMaxCand candidates,
// idx_map = their indices) draws from the same distribution with the same uniform.
constexpr int kPreselSlice = 8192;

__global__ void __launch_bounds__(kSampleThreads) sample_presel_kernel(
    float* __restrict__ cand_v, int* __restrict__ cand_i, const float* __restrict__ logits, int V, long ld,
    const float* __restrict__ temps, const int* __restrict__ top_ks, int per) {
  __shared__ float sl[kPreselSlice];
  __shared__ uint32_t hist[256];
  __shared__ uint32_t s_prefix, s_remaining, s_cnt_gt, s_cnt_eq;
  const int s = blockIdx.x, row_id = blockIdx.y, S = gridDim.x;
  const int j0 = s * per, len = max(0, min(per, V - j0));
  const size_t base = ((size_t)row_id * S + s) * kMaxCand;
  const float* row = logits + row_id * ld + j0;
  for (int j = threadIdx.x; j < len; j += blockDim.x) sl[j] = row[j];
  int K = top_ks[row_id];
  // greedy row: its slice max is all stage 2 needs; full-vocabulary rows (top_k = 0 or > kMaxCand)
  // are drawn by sample_full_kernel from the row itself, stage 2 skips them
  if (temps[row_id] <= 0.f || K <= 0 || K > kMaxCand) K = 1;
  if (K > len) K = len;
  __syncthreads();
  uint32_t prefix = 0, mask = 0, remaining = (uint32_t)K;
  for (int shift = 24; shift >= 0 && K > 0; shift -= 8) {
    for (int b = threadIdx.x; b < 256; b += blockDim.x) hist[b] = 0;
    __syncthreads();
    for (int j = threadIdx.x; j < len; j += blockDim.x) {
      const uint32_t k = fkey(sl[j]);
      if ((k & mask) == prefix) atomicAdd(&hist[(k >> shift) & 0xff], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t above = 0;
      int d = 255;
      for (; d > 0; --d) {
        if (above + hist[d] >= remaining) break;
        above += hist[d];
      }
      s_prefix = prefix | ((uint32_t)d << shift);
      s_remaining = remaining - above;
    }
    __syncthreads();
    prefix = s_prefix;
    remaining = s_remaining;
    mask |= 0xffu << shift;
  }
  if (threadIdx.x == 0) { s_cnt_gt = 0; s_cnt_eq = 0; }
  __syncthreads();
  const uint32_t n_gt = K > 0 ? (uint32_t)K - remaining : 0;
  for (int j = threadIdx.x; j < len && K > 0; j += blockDim.x) {
    const float x = sl[j];
    const uint32_t k = fkey(x);
    if (k > prefix) {
      const uint32_t p = atomicAdd(&s_cnt_gt, 1u);
      if (p < n_gt) { cand_v[base + p] = x; cand_i[base + p] = j0 + j; }
    } else if (k == prefix) {
      const uint32_t p = atomicAdd(&s_cnt_eq, 1u);
      if (p < remaining) { cand_v[base + n_gt + p] = x; cand_i[base + n_gt + p] = j0 + j; }
    }
  }
  for (int j = max(K, 0) + threadIdx.x; j < kMaxCand; j += blockDim.x) {
    cand_v[base + j] = -INFINITY;
    cand_i[base + j] = 0x7fffffff;
  }
}

// ---- full-vocabulary draw: top_k = 0 (or top_k > kMaxCand) -------------------------------
// The candidate kernels above draw from the top <= kMaxCand logits; a row without a top-k bound
// must draw from the softmax over the WHOLE vocabulary (with top-p: its nucleus over the full
// mass).  One workgroup per row, every pass a sweep over the row (L2-resident after the first):
//   1. row max (argmax pass);
//   2. top_k > kMaxCand: the K-th largest key by an exact 4 x 8-bit radix count select (members:
//      keys >= it; ties at the K-th value all kept);
//   3. top_p < 1: the nucleus threshold by a radix select on MASS instead of count: 4 passes of
//      256-bucket histograms of the members' fixed-point weights w = exp((l - max) / T) * 2^40
//      (u64 LDS atomics: integer sums, so the result does not depend on the order in which the
//      threads add -- a seeded request draws the same token every time); the threshold key's
//      ties are taken in vocabulary order until the mass reaches p of the total;
//   4. the draw: inverse CDF over the nucleus in VOCABULARY order (any fixed order gives the
//      same distribution), each thread owning one contiguous chunk: per-thread tie counts and
//      masses, two block scans, and the thread whose mass interval holds u * total walks its chunk.
// Weights below 2^-40 of the max's round to 0 (<= V * 2^-40 ~ 1e-7 of the mass for a 128k vocab).
constexpr float kFixOne = 1099511627776.0f;  // 2^40: the row max's fixed-point weight

__device__ __forceinline__ unsigned long long fix_w(float x, float vmax, float invT) {
  return (unsigned long long)(__expf((x - vmax) * invT) * kFixOne);
}

__device__ __forceinline__ float key_float(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

__global__ void __launch_bounds__(kSampleThreads) sample_full_kernel(
    long* __restrict__ out, const float* __restrict__ logits, int V, long ld, const float* __restrict__ temps,
    const int* __restrict__ top_ks, const float* __restrict__ top_ps, const float* __restrict__ uniform) {
  __shared__ unsigned long long hm[256];
  __shared__ uint32_t hc[256];
  __shared__ unsigned long long tm[kSampleThreads];
  __shared__ uint32_t tcnt[kSampleThreads];
  __shared__ float sv[kSampleThreads / 64];
  __shared__ int si[kSampleThreads / 64];
  __shared__ uint32_t s_prefix, s_rem;
  __shared__ unsigned long long s_need, s_total;

  const int row_id = blockIdx.x, tid = threadIdx.x;
  const float T = temps[row_id];
  const int K = top_ks[row_id];
  if (T <= 0.f || (K > 0 && K <= kMaxCand)) return;  // sample_kernel's rows
  const float* row = logits + row_id * ld;
  float vmax;
  int imax;
  block_argmax(row, V, sv, si, vmax, imax);
  const float invT = 1.f / T;

  // 2. members: keys >= thr_k
  uint32_t thr_k = 0;
  if (K > 0 && K < V) {
    uint32_t prefix = 0, mask = 0, remaining = (uint32_t)K;
    for (int shift = 24; shift >= 0; shift -= 8) {
      for (int b = tid; b < 256; b += blockDim.x) hc[b] = 0;
      __syncthreads();
      for (int j = tid; j < V; j += blockDim.x) {
        const uint32_t k = fkey(row[j]);
        if ((k & mask) == prefix) atomicAdd(&hc[(k >> shift) & 0xff], 1u);
      }
      __syncthreads();
      if (tid == 0) {
        uint32_t above = 0;
        int d = 255;
        for (; d > 0; --d) {
          if (above + hc[d] >= remaining) break;
          above += hc[d];
        }
        s_prefix = prefix | ((uint32_t)d << shift);
        s_rem = remaining - above;
      }
      __syncthreads();
      prefix = s_prefix;
      remaining = s_rem;
      mask |= 0xffu << shift;
    }
    thr_k = prefix;
  }

  // 3. nucleus: keys > thr, plus the first n_eq keys == thr in vocabulary order
  uint32_t thr = thr_k, n_eq = 0xffffffffu;
  const float p = top_ps[row_id];
  if (p < 1.f) {
    uint32_t prefix = 0, mask = 0;
    for (int shift = 24; shift >= 0; shift -= 8) {
      for (int b = tid; b < 256; b += blockDim.x) { hm[b] = 0; hc[b] = 0; }
      __syncthreads();
      for (int j = tid; j < V; j += blockDim.x) {
        const float x = row[j];
        const uint32_t k = fkey(x);
        if (k >= thr_k && (k & mask) == prefix) {
          const uint32_t d = (k >> shift) & 0xff;
          atomicAdd(&hm[d], fix_w(x, vmax, invT));
          atomicAdd(&hc[d], 1u);
        }
      }
      __syncthreads();
      if (tid == 0) {
        unsigned long long need;
        if (shift == 24) {
          unsigned long long tot = 0;
          for (int b = 0; b < 256; ++b) tot += hm[b];
          need = (unsigned long long)ceil((double)p * (double)tot);
          if (need == 0) need = 1;
        } else {
          need = s_need;
        }
        unsigned long long above = 0;
        int d = 255;
        for (; d > 0; --d) {
          if (above + hm[d] >= need) break;
          above += hm[d];
        }
        s_prefix = prefix | ((uint32_t)d << shift);
        s_need = need > above ? need - above : 1;
        s_rem = hc[d];
      }
      __syncthreads();
      prefix = s_prefix;
      mask |= 0xffu << shift;
    }
    thr = prefix;
    const unsigned long long wt = fix_w(key_float(thr), vmax, invT);
    n_eq = s_rem;
    if (wt > 0) {
      const unsigned long long t = (s_need + wt - 1) / wt;
      if (t < n_eq) n_eq = (uint32_t)(t < 1 ? 1 : t);
    }
  }

  // 4. the draw, vocabulary order
  const int ch = (V + (int)blockDim.x - 1) / (int)blockDim.x;
  const int j0 = min(V, tid * ch), j1 = min(V, j0 + ch);
  uint32_t ties = 0;
  for (int j = j0; j < j1; ++j) ties += fkey(row[j]) == thr;
  tcnt[tid] = ties;
  __syncthreads();
  if (tid == 0) {
    uint32_t acc = 0;
    for (int t = 0; t < (int)blockDim.x; ++t) { const uint32_t v = tcnt[t]; tcnt[t] = acc; acc += v; }
  }
  __syncthreads();
  const uint32_t tie0 = tcnt[tid];
  unsigned long long m = 0;
  uint32_t tr = tie0;
  for (int j = j0; j < j1; ++j) {
    const float x = row[j];
    const uint32_t k = fkey(x);
    const bool in = k > thr || (k == thr && tr++ < n_eq);
    if (in) m += fix_w(x, vmax, invT);
  }
  tm[tid] = m;
  __syncthreads();
  if (tid == 0) {
    unsigned long long acc = 0;
    for (int t = 0; t < (int)blockDim.x; ++t) { const unsigned long long v = tm[t]; tm[t] = acc; acc += v; }
    s_total = acc;
  }
  __syncthreads();
  const unsigned long long total = s_total;
  unsigned long long target = (unsigned long long)((double)uniform[row_id] * (double)total);
  if (target >= total) target = total > 0 ? total - 1 : 0;
  const unsigned long long base = tm[tid];
  if (total == 0) {
    if (tid == 0) out[row_id] = imax == 0x7fffffff ? 0 : imax;
    return;
  }
  if (m > 0 && base <= target && target < base + m) {
    unsigned long long cum = base;
    tr = tie0;
    int pick = j1 - 1;
    for (int j = j0; j < j1; ++j) {
      const float x = row[j];
      const uint32_t k = fkey(x);
      const bool in = k > thr || (k == thr && tr++ < n_eq);
      if (!in) continue;
      cum += fix_w(x, vmax, invT);
      if (cum > target) { pick = j; break; }
    }
    out[row_id] = pick;
  }
}

// workgroups per row of the pre-selection (1 = sample_kernel alone over the full row)
int sample_splits(int n, int V) {
  if (n <= 0 || n >= 64) return 1;
  const int need = (V + kPreselSlice - 1) / kPreselSlice;  // slices must fit LDS
  const int S = std::max(need, std::min(16, (256 + n - 1) / n));
  return S <= 1 ? 1 : S;
}

void launch_argmax(long* out, const float* logits, int n, int V, long ld, hipStream_t st) {
  if (n == 0) return;
  argmax_kernel<<<n, kSampleThreads, 0, st>>>(out, logits, V, ld);
}

// workgroups per row: enough to put ~256 workgroups on the chip, >= 2 16-B loads per thread
int argmax_splits(int n, int V) {
  if (n <= 0 || n >= 128) return 1;
  const int by_size = V / (8 * kSampleThreads * 2);
  return std::max(1, std::min({64, by_size, (256 + n - 1) / n}));
}

void launch_argmax_bf16(long* out, const void* logits, int n, int V, long ld, void* ws, hipStream_t st) {
  if (n == 0) return;
  const int S = ws ? argmax_splits(n, V) : 1;
  if (S <= 1) {
    argmax_bf16_kernel<<<n, kSampleThreads, 0, st>>>(out, (const uint16_t*)logits, V, ld);
    return;
  }
  auto* keys = (unsigned long long*)ws;
  argmax_bf16_split_kernel<<<dim3(S, n), kSampleThreads, 0, st>>>(keys, (const uint16_t*)logits, V, ld, S);
  argmax_keys_kernel<<<n, 64, 0, st>>>(out, keys, S);
}

void launch_sample(long* out, const float* logits, int n, int V, long ld, const float* temps,
                   const int* top_ks, const float* top_ps, const float* uniform, void* ws, bool full,
                   hipStream_t st) {
  if (n == 0) return;
  // rows with top_k = 0 / > kMaxCand (the caller knows whether there are any): drawn from the
  // whole row; the candidate kernels below skip them
  if (full) sample_full_kernel<<<n, kSampleThreads, 0, st>>>(out, logits, V, ld, temps, top_ks, top_ps, uniform);
  const int S = ws ? sample_splits(n, V) : 1;
  if (S <= 1) {
    sample_kernel<<<n, kSampleThreads, 0, st>>>(out, logits, V, ld, temps, top_ks, top_ps, uniform);
    return;
  }
  const int per = (V + S - 1) / S;
  const long C = (long)S * kMaxCand;  // candidates per row
  auto* cv = (float*)ws;
  auto* ci = (int*)((char*)ws + (size_t)n * C * sizeof(float));
  sample_presel_kernel<<<dim3(S, n), kSampleThreads, 0, st>>>(cv, ci, logits, V, ld, temps, top_ks, per);
  sample_kernel<<<n, kSampleThreads, 0, st>>>(out, cv, (int)C, C, temps, top_ks, top_ps, uniform, ci);
}

long sample_workspace_bytes(int n, int V) {
  const int S = sample_splits(n, V);
  return S <= 1 ? 0 : (long)n * S * kMaxCand * (sizeof(float) + sizeof(int));
}

}  // namespace mlop
