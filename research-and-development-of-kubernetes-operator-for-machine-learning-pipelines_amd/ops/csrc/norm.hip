// RMSNorm (K3) and fused residual-add + RMSNorm for gfx950.
//
// One workgroup per token row; every thread keeps VPT 16-byte vectors of the
// row in registers, so the row is read from HBM exactly once and written once
// (memory-bound: the target is the HBM roof, cdna_hip_programming.md App. B
// "Element-wise"/"Reduction").  Residual-add semantics follow the Llama
// decoder: residual <- bf16(residual + x); y <- bf16(rms(residual) * w).
#include "common.h"
#include "launch.h"

namespace mlop {

template <int VPT, bool ADD>
__global__ void __launch_bounds__(1024) rmsnorm_kernel(uint16_t* __restrict__ out,
                                                      uint16_t* __restrict__ residual,
                                                      const uint16_t* __restrict__ x,
                                                      const uint16_t* __restrict__ w, float eps,
                                                      int H) {
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  const int nvec = H >> 3;
  const size_t base = (size_t)row * H;
  float v[VPT][8];
  float ss = 0.f;
  // the norm weights are loaded with the row, not after the reduction (no dependent round trip
  // after it; at batch 1 the launch stayed 4.7 us either way, scripts/history/r4_norm1.sh)
  u32x4 wv[VPT];
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int vi = threadIdx.x + i * blockDim.x;
    wv[i] = vi < nvec ? *reinterpret_cast<const u32x4*>(w + vi * 8) : u32x4{0, 0, 0, 0};
  }
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int vi = threadIdx.x + i * blockDim.x;
    if (vi < nvec) {
      u32x4 a = *reinterpret_cast<const u32x4*>(x + base + vi * 8);
      if constexpr (ADD) {
        u32x4 r = *reinterpret_cast<const u32x4*>(residual + base + vi * 8);
        u32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          // round the sum to bf16 exactly as the bf16 residual stream does
          float s0 = lo_bf(a[j]) + lo_bf(r[j]);
          float s1 = hi_bf(a[j]) + hi_bf(r[j]);
          o[j] = pack2(s0, s1);
          v[i][2 * j] = lo_bf(o[j]);
          v[i][2 * j + 1] = hi_bf(o[j]);
        }
        *reinterpret_cast<u32x4*>(residual + base + vi * 8) = o;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[i][2 * j] = lo_bf(a[j]);
          v[i][2 * j + 1] = hi_bf(a[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  ss = block_sum(ss, scratch);
  const float inv = rsqrtf(ss / (float)H + eps);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int vi = threadIdx.x + i * blockDim.x;
    if (vi < nvec) {
      u32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        // HF LlamaRMSNorm: weight * bf16(x * inv)
        float a0 = bf2f(f2bf(v[i][2 * j] * inv)) * lo_bf(wv[i][j]);
        float a1 = bf2f(f2bf(v[i][2 * j + 1] * inv)) * hi_bf(wv[i][j]);
        o[j] = pack2(a0, a1);
      }
      *reinterpret_cast<u32x4*>(out + base + vi * 8) = o;
    }
  }
}

// Wave-per-row form for the many-row passes (H = 512 * VPL): each lane issues all
// of its row's 16-B loads up front and the sum of squares is one wave reduction,
// so there is no LDS and no barrier, and a CU keeps several rows per SIMD in
// flight instead of one 8-wave row per quarter CU (the block form above waits on
// one 32 KB row's round trip per workgroup).
template <int VPL, bool ADD>
__global__ void __launch_bounds__(256) rmsnorm_wave_kernel(uint16_t* __restrict__ out,
                                                           uint16_t* __restrict__ residual,
                                                           const uint16_t* __restrict__ x,
                                                           const uint16_t* __restrict__ w,
                                                           float eps, int M, int H) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;  // whole wave; no barrier below
  const size_t base = (size_t)row * H;
  u32x4 a[VPL], wv[VPL];
#pragma unroll
  for (int i = 0; i < VPL; ++i) a[i] = *reinterpret_cast<const u32x4*>(x + base + (lane + i * 64) * 8);
#pragma unroll
  for (int i = 0; i < VPL; ++i) wv[i] = *reinterpret_cast<const u32x4*>(w + (lane + i * 64) * 8);  // with the row
  if constexpr (ADD) {
    u32x4 r[VPL];
#pragma unroll
    for (int i = 0; i < VPL; ++i)
      r[i] = *reinterpret_cast<const u32x4*>(residual + base + (lane + i * 64) * 8);
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j)  // bf16-rounded sum, as the residual stream stores it
        a[i][j] = pack2(lo_bf(a[i][j]) + lo_bf(r[i][j]), hi_bf(a[i][j]) + hi_bf(r[i][j]));
      *reinterpret_cast<u32x4*>(residual + base + (lane + i * 64) * 8) = a[i];
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float lo = lo_bf(a[i][j]), hi = hi_bf(a[i][j]);
      ss += lo * lo + hi * hi;
    }
  ss = wave_sum(ss);
  const float inv = rsqrtf(ss / (float)H + eps);
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j)  // HF LlamaRMSNorm: weight * bf16(x * inv)
      o[j] = pack2(bf2f(f2bf(lo_bf(a[i][j]) * inv)) * lo_bf(wv[i][j]),
                   bf2f(f2bf(hi_bf(a[i][j]) * inv)) * hi_bf(wv[i][j]));
    *reinterpret_cast<u32x4*>(out + base + (lane + i * 64) * 8) = o;
  }
}

// fewer rows: the block form's 8-wave fan-out per row wins (at batch 1 the wave form measured
// 345 vs 351 tok/s, scripts/history INDEX r4_norm1)
constexpr int kWaveRowsMinM = 256;

template <bool ADD>
static bool dispatch_wave(uint16_t* out, uint16_t* residual, const uint16_t* x, const uint16_t* w,
                          float eps, int M, int H, hipStream_t st) {
  if (M < kWaveRowsMinM || H % 512) return false;
  const int g = cdiv(M, 4);
  switch (H / 512) {
    case 1: rmsnorm_wave_kernel<1, ADD><<<g, 256, 0, st>>>(out, residual, x, w, eps, M, H); return true;
    case 2: rmsnorm_wave_kernel<2, ADD><<<g, 256, 0, st>>>(out, residual, x, w, eps, M, H); return true;
    case 4: rmsnorm_wave_kernel<4, ADD><<<g, 256, 0, st>>>(out, residual, x, w, eps, M, H); return true;
    case 8: rmsnorm_wave_kernel<8, ADD><<<g, 256, 0, st>>>(out, residual, x, w, eps, M, H); return true;
    case 16: rmsnorm_wave_kernel<16, ADD><<<g, 256, 0, st>>>(out, residual, x, w, eps, M, H); return true;
    default: return false;
  }
}

template <bool ADD>
static void dispatch(uint16_t* out, uint16_t* residual, const uint16_t* x, const uint16_t* w,
                     float eps, int M, int H, hipStream_t st) {
  if (dispatch_wave<ADD>(out, residual, x, w, eps, M, H, st)) return;
  const int nvec = H / 8;
  int vpt = 1;
  while (vpt < 8 && nvec / vpt > 512) vpt <<= 1;
  int threads = ((cdiv(nvec, vpt) + 63) / 64) * 64;
  if (M == 0) return;
  switch (vpt) {
    case 1: rmsnorm_kernel<1, ADD><<<M, threads, 0, st>>>(out, residual, x, w, eps, H); break;
    case 2: rmsnorm_kernel<2, ADD><<<M, threads, 0, st>>>(out, residual, x, w, eps, H); break;
    case 4: rmsnorm_kernel<4, ADD><<<M, threads, 0, st>>>(out, residual, x, w, eps, H); break;
    default: rmsnorm_kernel<8, ADD><<<M, threads, 0, st>>>(out, residual, x, w, eps, H); break;
  }
}

void launch_rmsnorm(void* out, const void* x, const void* w, float eps, int M, int H,
                    hipStream_t st) {
  dispatch<false>((uint16_t*)out, nullptr, (const uint16_t*)x, (const uint16_t*)w, eps, M, H, st);
}

void launch_add_rmsnorm(void* out, void* residual, const void* x, const void* w, float eps, int M,
                        int H, hipStream_t st) {
  dispatch<true>((uint16_t*)out, (uint16_t*)residual, (const uint16_t*)x, (const uint16_t*)w, eps,
                 M, H, st);
}

}  // namespace mlop
