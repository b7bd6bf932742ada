// Element-wise / gather kernels: SiLU-and-mul (K8) and embedding row gather (K9).
// Memory-bound: 16-byte vectors per lane, grid-stride (cdna_hip_programming.md Guideline 11/13).
#include "common.h"
#include "launch.h"

namespace mlop {

// out[m, i] = silu(gate_i) * up_i of the fused gate_up projection output x[m, 2I]:
//   interleaved = 0: x = [gate | up];  interleaved = 1: groups of 16 (g0..15, u0..15, ...)
__global__ void __launch_bounds__(256) silu_mul_kernel(uint16_t* __restrict__ out,
                                                      const uint16_t* __restrict__ x, int M, int I,
                                                      int interleaved) {
  const int vpr = I >> 3;
  const long total = (long)M * vpr;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const long m = idx / vpr;
    const int c = (int)(idx % vpr) * 8;
    const uint16_t* row = x + m * 2 * (long)I;
    const int gc = interleaved ? (c / 16) * 32 + (c % 16) : c;
    const int uc = interleaved ? gc + 16 : I + c;
    u32x4 g = *reinterpret_cast<const u32x4*>(row + gc);
    u32x4 u = *reinterpret_cast<const u32x4*>(row + uc);
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      // HF computes silu in bf16 then multiplies in bf16: round after silu
      float g0 = lo_bf(g[j]), g1 = hi_bf(g[j]);
      float s0 = bf2f(f2bf(g0 * __builtin_amdgcn_rcpf(1.f + __expf(-g0))));
      float s1 = bf2f(f2bf(g1 * __builtin_amdgcn_rcpf(1.f + __expf(-g1))));
      o[j] = pack2(s0 * lo_bf(u[j]), s1 * hi_bf(u[j]));
    }
    *reinterpret_cast<u32x4*>(out + m * (long)I + c) = o;
  }
}

void launch_silu_mul(void* out, const void* x, int M, int I, int interleaved, hipStream_t st) {
  if (M == 0) return;
  const long total = (long)M * (I / 8);
  int grid = (int)std::min<long>((total + 255) / 256, 2048);
  silu_mul_kernel<<<grid, 256, 0, st>>>((uint16_t*)out, (const uint16_t*)x, M, I, interleaved);
}

// out[t, :] = table[ids[t] - vocab_start, :] if the id is in this rank's vocab shard, else 0
// (vocab-parallel embedding: the zero rows are summed away by the TP all-reduce).
__global__ void __launch_bounds__(256) embedding_kernel(uint16_t* __restrict__ out,
                                                       const uint16_t* __restrict__ table,
                                                       const long* __restrict__ ids, int H,
                                                       long vocab_start, long vocab_end) {
  const int t = blockIdx.x;
  const long id = ids[t];
  const bool in = id >= vocab_start && id < vocab_end;
  const uint16_t* src = table + (in ? (id - vocab_start) : 0) * (long)H;
  uint16_t* dst = out + (long)t * H;
  for (int c = threadIdx.x * 8; c < H; c += blockDim.x * 8) {
    u32x4 v = in ? *reinterpret_cast<const u32x4*>(src + c) : u32x4{0, 0, 0, 0};
    *reinterpret_cast<u32x4*>(dst + c) = v;
  }
}

void launch_embedding(void* out, const void* table, const long* ids, int T, int H, long vocab_start,
                      long vocab_end, hipStream_t st) {
  if (T == 0) return;
  embedding_kernel<<<T, 256, 0, st>>>((uint16_t*)out, (const uint16_t*)table, ids, H, vocab_start,
                                      vocab_end);
}

// Fault injection only (MLOP_INJECT_STEP_DEVICE_US, runtime/engine.py): one wave that waits until
// the constant-rate wall clock has advanced `ticks`, so an engine step gets slower ON THE DEVICE
// alone (the host stays idle) -- the canary test of the GPU-side TPOT guard.  Always terminates.
__global__ void __launch_bounds__(64) device_delay_kernel(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(16);
}

void launch_device_delay(long long ticks, hipStream_t st) {
  if (ticks <= 0) return;
  device_delay_kernel<<<1, 64, 0, st>>>(ticks);
}

}  // namespace mlop
