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

// Cross-lane all-reduces without the LDS: __shfl_xor lowers to ds_bpermute_b32 (an LDS
// round trip, ~50+ cycles on the reduction's critical path per step).  Here the steps
// inside a 16-lane row are DPP operand modifiers (quad_perm [1,0,3,2] / [2,3,0,1],
// row_half_mirror, row_mirror: each pairs every lane with one from the other half of its
// group), and the 16- / 32-lane steps are gfx950's v_permlane16/32_swap.  Each step
// combines x with its partner's y while the partner combines y with x: commutative ops give
// every lane bit-identical results.
namespace detail {
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
}  // namespace detail

// sum / max over lane groups {l, l^16, l^32, l^48} (the 4 lane groups of an MFMA fragment
// column).  The swap leaves (self, partner) in (r[0], r[1]) on one side and (partner, self) on
// the other, so combining r[0] with r[1] needs no lane select.
__device__ __forceinline__ float sum_x16_x32(float v) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float max_x16_x32(float v) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

__device__ __forceinline__ float wave_sum(float v) {
  v += detail::dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += detail::dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += detail::dpp<0x141>(v);  // row_half_mirror: lane i <-> 7-i (the other quad)
  v += detail::dpp<0x140>(v);  // row_mirror: lane i <-> 15-i (the other 8 lanes)
  return sum_x16_x32(v);
}

__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, detail::dpp<0xB1>(v));
  v = fmaxf(v, detail::dpp<0x4E>(v));
  v = fmaxf(v, detail::dpp<0x141>(v));
  v = fmaxf(v, detail::dpp<0x140>(v));
  return max_x16_x32(v);
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

// SiLU of a bf16-rounded gate, rounded to bf16 (the GEMM epilogues' rounding).  The quotient
// is v_rcp_f32 x v_mul (1 ulp reciprocal, invisible after the bf16 rounding): an
// IEEE '/' expands to a ~10-instruction div_scale / div_fmas / div_fixup sequence, which in the
// four-wave GEMM's SiLU-mul epilogue (128 quotients per lane per tile, nothing to overlap
// with) was several microseconds per tile.  Large negative gates: exp -> inf, rcp -> 0, -0.
__device__ __forceinline__ float silu_bf(float g) {
  const float gb = bf2f(f2bf(g));
  return bf2f(f2bf(gb * __builtin_amdgcn_rcpf(1.f + __expf(-gb))));
}

__host__ __device__ constexpr int cdiv(int a, int b) { return (a + b - 1) / b; }

}  // namespace mlop
