// Shared device helpers for the gfx950 (CDNA4) kernels of the serving runtime.
//
// Conventions (all kernels):
//   * wave = 64 lanes; block sizes are multiples of 64.
//   * bf16 tensors are moved as 16-byte vectors (8 x bf16) wherever the row
//     length allows it (cdna_hip_programming.md Guideline 13).
//   * math in fp32, one rounding to bf16 on store (plain cast lowers to
//     v_cvt_pk_bf16_f32 and keeps NaNs NaN: MI355X_MICROARCH.md "Correctness boundaries").
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mlop {

using bf16x8 = __attribute__((ext_vector_type(8))) short;   // 16 B: one MFMA A/B fragment
using bf16x4 = __attribute__((ext_vector_type(4))) short;   // 8 B
using f32x4 = __attribute__((ext_vector_type(4))) float;    // 16x16 MFMA accumulator
using u32x4 = __attribute__((ext_vector_type(4))) uint32_t;
using u32x2 = __attribute__((ext_vector_type(2))) uint32_t;

typedef __attribute__((address_space(3))) void lds_void_t;  // LDS-DMA destination

// s_barrier without __syncthreads' fence (whose vmcnt(0) would drain in-flight
// LDS-DMA; cdna_hip_programming.md "Pipelining across barriers")
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ float bf2f_s(short v) { return bf2f((uint16_t)v); }

__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}

// pack two floats into one dword of two bf16 (lo in bits 0..15)
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

__device__ __forceinline__ float lo_bf(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi_bf(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum; `scratch` needs blockDim.x/64 floats. Result valid in all threads.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += scratch[i];
  __syncthreads();
  return t;
}

// MFMA 16x16x32 bf16 -> f32. Lane l holds A[row l&15][k 8(l>>4)+j] and
// B[k 8(l>>4)+j][col l&15]; C/D: col = l&15, row = 4(l>>4)+i
// (cdna_hip_programming.md §3 "Fragment layout").
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// SiLU of a bf16-rounded gate, rounded to bf16 (the GEMM epilogues' rounding)
__device__ __forceinline__ float silu_bf(float g) {
  const float gb = bf2f(f2bf(g));
  return bf2f(f2bf(gb / (1.f + __expf(-gb))));
}

__host__ __device__ constexpr int cdiv(int a, int b) { return (a + b - 1) / b; }

}  // namespace mlop
