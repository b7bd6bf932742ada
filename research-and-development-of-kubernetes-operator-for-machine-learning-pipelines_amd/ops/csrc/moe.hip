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
