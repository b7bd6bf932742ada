// Read-bandwidth microbench: how the per-instruction access shape of a weight stream affects
// HBM throughput on MI355X.  W [N][K] bf16 (K = 4096, 8 KiB rows), rotated over enough copies
// (> 1 GiB) that no pass hits L2 / MALL.  Every variant: 256-thread workgroups, each wave owns
// 32 rows x a K quarter (like a decode GEMM's weight tile), 8 x 16-B loads per lane per step in
// flight (U steps), nontemporal, summed into a sink so nothing is dead.  Shapes of ONE
// wave-instruction (1 KiB):
//   0: 16 rows x 64 B   (a v_mfma 16x16x32 B fragment loaded straight from memory)
//   1:  8 rows x 128 B  (the LDS-DMA tile piece of gemm.hip)
//   2:  2 rows x 512 B
//   3:  1 row  x 1 KiB  (the GEMV)
// Build: hipcc -O3 --offload-arch=gfx950 scripts/bw_shapes.hip -o build/bw_shapes
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

using u32x4 = __attribute__((ext_vector_type(4))) uint32_t;

template <int SHAPE, int U, int RPW = 32>
__global__ void __launch_bounds__(256) stream(const uint16_t* __restrict__ W, int N, int K, float* sink) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int row0 = blockIdx.x * RPW;  // RPW rows per workgroup, the 4 waves split K in quarters
  const int kq = K / 4, k0 = w * kq;
  // lane -> (row offset, element offset) inside one 1-KiB instruction
  int rr, ce;
  if (SHAPE == 0) { rr = lane & 15; ce = (lane >> 4) * 8; }          // 16 rows x 32 elements
  else if (SHAPE == 1) { rr = lane >> 3; ce = (lane & 7) * 8; }      // 8 rows x 64
  else if (SHAPE == 2) { rr = lane >> 5; ce = (lane & 31) * 8; }     // 2 rows x 256
  else { rr = 0; ce = lane * 8; }                                    // 1 row x 512
  constexpr int RPI = SHAPE == 0 ? 16 : SHAPE == 1 ? 8 : SHAPE == 2 ? 2 : 1;  // rows per instruction
  constexpr int EPI = 512 / RPI;                                      // elements per row per instr.
  // a step = 8 instructions; with more than 8 row groups (2 x 512 B, 1 KiB) consecutive steps
  // take the next 8 row groups before K advances (NB blocks)
  constexpr int RG = RPW / RPI > 0 ? RPW / RPI : 1;
  constexpr int IPRG = RG >= 8 ? 1 : 8 / RG;  // instructions per row group per step
  static_assert(RPW % RPI == 0, "rows per workgroup");
  constexpr int NB = RG >= 8 ? RG / 8 : 1;
  constexpr int step_k = IPRG * EPI;
  const int nsteps = NB * (kq / step_k);
  auto addr = [&](int i, int s) {
    const int b = s % NB, ks = s / NB;
    const int rg = RG >= 8 ? b * 8 + i : i / IPRG, ii = RG >= 8 ? 0 : i % IPRG;
    return reinterpret_cast<const u32x4*>(W + (size_t)(row0 + rg * RPI + rr) * K + k0 + ks * step_k + ii * EPI + ce);
  };
  u32x4 acc = {0, 0, 0, 0};
  u32x4 buf[U][8];
  auto load = [&](int slot, int s) {
#pragma unroll
    for (int i = 0; i < 8; ++i) buf[slot][i] = __builtin_nontemporal_load(addr(i, s));
  };
#pragma unroll
  for (int u = 0; u < U - 1; ++u) {
    load(u, u);
    __builtin_amdgcn_sched_barrier(0);
  }
  int s0 = 0;
  for (; s0 + 2 * U - 2 < nsteps; s0 += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      load((u + U - 1) % U, s0 + u + U - 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc ^= buf[u][i];
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  for (int s = s0; s < nsteps; ++s) {
    u32x4 t[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = __builtin_nontemporal_load(addr(i, s));
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= t[i];
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = 1.f;
}

template <int SHAPE, int U, int RPW = 32>
float run(const std::vector<uint16_t*>& ws, int N, int K, float* sink) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(a);
    for (auto* w : ws) stream<SHAPE, U, RPW><<<N / RPW, 256>>>(w, N, K, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    best = ms < best ? ms : best;
  }
  const double bytes = (double)N * K * 2 * ws.size();
  return (float)(bytes / (best * 1e-3) / 1e12);
}

int main() {
  for (int K : {4096, 14336}) {
    for (int N : {28672, 6144, 4096}) {
      if (K == 14336 && N != 4096) continue;
      const size_t one = (size_t)N * K * 2;
      const int copies = (int)((size_t)(1536u << 20) / one) + 1;
      std::vector<uint16_t*> ws(copies);
      for (auto& w : ws) {
        hipMalloc(&w, one);
        hipMemset(w, 0x3c, one);
      }
      float* sink;
      hipMalloc(&sink, 4096);
      run<0, 3>(ws, N, K, sink);  // warm
      printf("N=%d K=%d copies=%d  TB/s: frag16x64B U3 %.2f U4 %.2f | piece8x128B U3 %.2f U4 %.2f | "
             "2x512B U3 %.2f U4 %.2f | 1x1KiB U3 %.2f U4 %.2f | 8 rows/WG: piece U3 %.2f U2 %.2f, 1KiB U3 %.2f | "
             "16 rows/WG piece U3 %.2f\n",
             N, K, copies, run<0, 3>(ws, N, K, sink), run<0, 4>(ws, N, K, sink), run<1, 3>(ws, N, K, sink),
             run<1, 4>(ws, N, K, sink), run<2, 3>(ws, N, K, sink), run<2, 4>(ws, N, K, sink),
             run<3, 3>(ws, N, K, sink), run<3, 4>(ws, N, K, sink), run<1, 3, 8>(ws, N, K, sink),
             run<1, 2, 8>(ws, N, K, sink), run<3, 3, 8>(ws, N, K, sink), run<1, 3, 16>(ws, N, K, sink));
      for (auto* w : ws) hipFree(w);
      hipFree(sink);
    }
  }
  return 0;
}
