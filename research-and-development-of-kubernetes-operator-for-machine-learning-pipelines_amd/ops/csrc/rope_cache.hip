// Fused RoPE (K4) + paged KV-cache write (K5).
//
// Input is the raw output of the QKV projection, one row per token:
//   qkv[t] = [ q (Hq*D) | k (Hkv*D) | v (Hkv*D) ]   (bf16)
// The kernel rotates q and k (HF "rotate_half" layout, host-precomputed
// cos/sin table: no on-device trig, cdna_hip_programming.md App. B) and
//   * writes q to q_out[t, Hq, D] (contiguous, the attention kernel's input);
//   * writes k to k_cache[block, Hkv, BS, D]   (token-major rows, the A operand of S^T = K.Q^T);
//   * writes v to v_cache[block, Hkv, BS, D]   (token-major rows too: attention.hip stages a
//     page pair in LDS and reads the A operand of O^T = V^T.P^T with ds_read_b64_tr_b16).
// slot[t] = block*BS + offset, or < 0 for padding tokens (no cache write).
#include "common.h"
#include "launch.h"

namespace mlop {

// SLABS: the input is the QKV projection's split-K partials instead of its bf16 output,
// ws[s][T][qkv_stride] fp32: the 8 values of a vector are summed over the splits and rounded
// to bf16 (splitk_reduce_kernel's order and rounding), so one launch replaces reduce + RoPE.
// f: the row's RMSNorm factor of the mid norm chain (1 otherwise), applied to the summed
// accumulators before the bf16 rounding (W4_RS's order)
template <bool SLABS>
__device__ __forceinline__ u32x4 load8(const uint16_t* row, const float* ws, int t, int T, int stride,
                                       int splits, int col, float f = 1.f) {
  if constexpr (!SLABS) {
    return *reinterpret_cast<const u32x4*>(row + col);
  } else {
    float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int s = 0; s < splits; ++s) {
      const float4* p = reinterpret_cast<const float4*>(ws + ((size_t)s * T + t) * stride + col);
      const float4 x = p[0], y = p[1];
      a[0] += x.x; a[1] += x.y; a[2] += x.z; a[3] += x.w;
      a[4] += y.x; a[5] += y.y; a[6] += y.z; a[7] += y.w;
    }
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = pack2(a[2 * j] * f, a[2 * j + 1] * f);
    return o;
  }
}

template <bool SLABS>
__global__ void __launch_bounds__(256) rope_cache_kernel(
    uint16_t* __restrict__ q_out, uint16_t* __restrict__ k_cache, uint16_t* __restrict__ v_cache,
    const uint16_t* __restrict__ qkv, const int* __restrict__ pos, const float* __restrict__ cos_sin,
    const int* __restrict__ slots, int Hq, int Hkv, int D, int qkv_stride, int BS,
    const float* __restrict__ ws = nullptr, int splits = 0, const float* __restrict__ ss_in = nullptr,
    float ss_inv_k = 0.f, float ss_eps = 0.f) {
  const int t = blockIdx.x, T = gridDim.x;
  const float f = SLABS && ss_in != nullptr ? rsqrtf(ss_in[t] * ss_inv_k + ss_eps) : 1.f;
  const int half = D >> 1;
  const int vph = half >> 3;  // 8-element vectors per half-head
  const int p = pos[t];
  const int slot = slots ? slots[t] : -1;
  const float* cs = cos_sin + (size_t)p * D;
  const uint16_t* row = SLABS ? nullptr : qkv + (size_t)t * qkv_stride;
  const int n_rope = (Hq + Hkv) * vph;
  const int n_v = Hkv * (D >> 3);
  const int blk = slot >= 0 ? slot / BS : 0;
  const int off = slot >= 0 ? slot % BS : 0;
  // gridDim.y blocks per token share its items (one item per thread at the decoder's head
  // counts: one dependent load chain each instead of two in a row)
  for (int it = threadIdx.x + blockIdx.y * blockDim.x; it < n_rope + n_v; it += blockDim.x * gridDim.y) {
    if (it < n_rope) {
      const int h = it / vph, c = (it % vph) * 8;
      // q heads then k heads are contiguous
      u32x4 a = load8<SLABS>(row, ws, t, T, qkv_stride, splits, h * D + c, f);
      u32x4 b = load8<SLABS>(row, ws, t, T, qkv_stride, splits, h * D + half + c, f);
      const float4* cp = reinterpret_cast<const float4*>(cs + c);
      const float4* sp = reinterpret_cast<const float4*>(cs + half + c);
      float4 c0 = cp[0], c1 = cp[1], s0 = sp[0], s1 = sp[1];
      float cc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
      float ss[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      u32x4 oa, ob;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float x0 = lo_bf(a[j]), x1 = hi_bf(a[j]);
        float y0 = lo_bf(b[j]), y1 = hi_bf(b[j]);
        oa[j] = pack2(x0 * cc[2 * j] - y0 * ss[2 * j], x1 * cc[2 * j + 1] - y1 * ss[2 * j + 1]);
        ob[j] = pack2(y0 * cc[2 * j] + x0 * ss[2 * j], y1 * cc[2 * j + 1] + x1 * ss[2 * j + 1]);
      }
      if (h < Hq) {
        uint16_t* dst = q_out + ((size_t)t * Hq + h) * D;
        *reinterpret_cast<u32x4*>(dst + c) = oa;
        *reinterpret_cast<u32x4*>(dst + half + c) = ob;
      } else if (slot >= 0) {
        const int kh = h - Hq;
        uint16_t* dst = k_cache + (((size_t)blk * Hkv + kh) * BS + off) * D;
        *reinterpret_cast<u32x4*>(dst + c) = oa;
        *reinterpret_cast<u32x4*>(dst + half + c) = ob;
      }
    } else if (slot >= 0) {
      const int iv = it - n_rope;
      const int kh = iv / (D >> 3), c = (iv % (D >> 3)) * 8;
      u32x4 a = load8<SLABS>(row, ws, t, T, qkv_stride, splits, (Hq + Hkv + kh) * D + c, f);
      *reinterpret_cast<u32x4*>(v_cache + (((size_t)blk * Hkv + kh) * BS + off) * D + c) = a;
    }
  }
}

void launch_rope_cache(void* q_out, void* k_cache, void* v_cache, const void* qkv, const int* pos,
                       const float* cos_sin, const int* slots, int T, int Hq, int Hkv, int D,
                       int qkv_stride, int BS, hipStream_t st) {
  if (T == 0) return;
  const int items = (Hq + Hkv) * (D / 16) + Hkv * (D / 8);  // 16-B vectors per token
  const int by = std::min(2, (items + 255) / 256);               // as launch_rope_cache_slabs
  rope_cache_kernel<false><<<dim3(T, by), 256, 0, st>>>((uint16_t*)q_out, (uint16_t*)k_cache, (uint16_t*)v_cache,
                                              (const uint16_t*)qkv, pos, cos_sin, slots, Hq, Hkv, D,
                                              qkv_stride, BS);
}

void launch_rope_cache_slabs(const RopeEpi& re, const float* ws, int splits, int T, int N, hipStream_t st) {
  if (T == 0) return;
  const int items = (re.Hq + re.Hkv) * 8 + re.Hkv * 16;  // 16-B vectors per token (head_dim 128)
  // two blocks per token when the items exceed one block (batch 16 / 64 +0.4 %, interleaved,
  // scripts/r5_ropesplit.sh)
  const int by = std::min(2, (items + 255) / 256);
  rope_cache_kernel<true><<<dim3(T, by), 256, 0, st>>>(re.q_out, re.k_cache, re.v_cache, nullptr, re.pos, re.cos_sin,
                                             re.slots, re.Hq, re.Hkv, 128, N, re.BS, ws, splits, re.ss_in,
                                             re.ss_inv_k, re.ss_eps);
}

}  // namespace mlop
