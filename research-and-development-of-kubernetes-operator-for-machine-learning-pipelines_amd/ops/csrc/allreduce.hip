// K15: one-shot all-reduce over xGMI peer memory (tensor-parallel decode).
//
// Why: a TP decode step all-reduces [B, hidden] bf16 twice per layer (8-16 KiB
// per token row); at these sizes RCCL's ring is latency-bound (2(N-1) hops).
// xGMI on MI355X is point-to-point (7 links per GPU), so ONE hop in which every
// rank reads all peers' inputs at once uses all links in parallel
// (SURVEY.md §2.5 K15 / §5 "distributed communication backend").
//
// Protocol (per rank: one IPC-exported buffer = flags | data[2]):
//   * every block b copies its slice of the input into its OWN buffer, then
//     (one lane, after every wave's vmcnt(0) + a block barrier) a SYSTEM-scope
//     release (L2 write-back) and a relaxed system-scope store of the epoch into
//     flag[rank][b] of EVERY peer's buffer;
//   * lanes 0..N-1 of wave 0 poll flag[p][b] of the local buffer until it
//     reaches the epoch (>=: a fast peer may already be one call ahead), then a
//     system-scope acquire, vmcnt(0) and a block barrier before any peer load
//     (MI355X_MICROARCH.md "Valid forms"; cdna_hip_programming.md Guideline 16);
//   * the block sums its slice over ranks 0..N-1 IN RANK ORDER in fp32 (every
//     rank produces bitwise-identical output) and stores bf16.
//   * epochs live in device memory, one counter per block, so the kernel is
//     hipGraph-capturable (no host-side state per call); data is double
//     buffered by epoch parity: a peer can run at most one call ahead (it
//     needs this rank's flag of the call in between), so the parity it
//     overwrites is never the one still being read.  The grid is FIXED
//     (kBlocks) so every block advances its epoch on every call.
//   * every poll is bounded: on timeout the block sets an error word (read by
//     car_error) and finishes — a wedged peer never hangs the GPU.
//
// Memory (two layouts, car_create's `split`):
//   * split = 0: ONE IPC-exported buffer, flags AND data, allocated UNCACHED
//     (hipExtMallocWithFlags(hipDeviceMallocUncached));
//   * split = 1: the flag banks alone in an uncached buffer, the data parities in a separate
//     ordinary (cached, coarse-grained) hipMalloc buffer, each IPC-exported.
// The flag lines are written by REMOTE agents: in coarse-grained memory this device's L2 may
// keep a stale copy of a flag line a peer rewrote, and a poll served from it would never see
// the epoch -- so flags are uncached in both layouts, as RCCL keeps its flags.  Data does not
// need that: every data line is published before a system-scope release (L2 write-back) that
// precedes its flag, and read after a system-scope acquire (L2 invalidate of non-local lines)
// that follows the flag poll, so a cached data buffer sees the same values.  What the layouts
// trade is bandwidth: uncached data keeps every publish / peer read at the memory side (no L2
// write combining, no L2 hits on the local copy), which is free for decode-sized messages but
// could be paid per byte on the two-shot kernel's 1-64 MiB prefill chunks.  Measured on one
// GPU (scripts/bench_car.py, profiles/r05_car_memory.md): the layouts are within -5 / +9 % at
// 1-64 MiB, and the uncached one is 11-23 % faster at 256 KiB-4 MiB one-shot messages, so
// split = 0 is the default (parallel/custom_ar.py SPLIT_DATA).  What bounds large messages is
// the fixed 64-workgroup grid (a 64 MiB two-shot call: 276 us vs 38 us for a plain copy on one
// GPU), which on a node keeps pace with the ~400 GB/s of xGMI read bandwidth per GPU.  If the driver refuses to IPC-export uncached memory the flags fall
// back to hipMalloc (car_mem_mode() reports which layout is in use).
#include "common.h"
#include "launch.h"

#include <cstring>
#include <stdexcept>
#include <string>

namespace mlop {

namespace {

constexpr int kMaxRanks = 8;
constexpr int kBlocks = 64;
constexpr int kThreads = 512;
constexpr int kFlagStride = 16;  // u32 per flag slot: one 64-B line per (source rank, block)
constexpr size_t kFlagBank = (size_t)kMaxRanks * kBlocks * kFlagStride * 4;
constexpr size_t kFlagsBytes = 2 * kFlagBank;  // bank 0: one-shot + two-shot phase 1; bank 1: two-shot phase 2
constexpr long kMaxSpins = 1L << 26;

struct Peers {
  uint8_t* base[kMaxRanks];  // flag banks (and, split = 0, the data parities after them)
  uint8_t* data[kMaxRanks];  // data parity 0 | parity 1 of each rank
};

struct CarState {
  int rank = 0, world = 1, device = 0;
  int uncached = 0;  // 1: the flag buffer is hipDeviceMallocUncached memory
  int split = 0;     // 1: data in its own cached buffer (dbuf), else after the flags in buf
  size_t max_bytes = 0;  // per parity
  uint8_t* buf = nullptr;
  uint8_t* dbuf = nullptr;
  uint32_t* epochs = nullptr;
  int* err = nullptr;       // device alias of err_host
  int* err_host = nullptr;
  Peers peers{};
};

#define CAR_CHECK(x)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess)                                                              \
      throw std::runtime_error(std::string("custom all-reduce: ") + #x + ": " +        \
                               hipGetErrorString(e_));                                 \
  } while (0)

__device__ __forceinline__ void add_bf16x8(float (&acc)[8], const uint4 v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    acc[2 * j] += __uint_as_float(w[j] << 16);
    acc[2 * j + 1] += __uint_as_float(w[j] & 0xffff0000u);
  }
}

// add_out: out is the residual stream, out = bf16(out + bf16(sum)) (norm.hip's add rounding;
// each element read and written by its one owning thread): the tensor-parallel decode norm
// chain's all-reduce + residual add in one launch (its consumers take their RMSNorm factors
// from the residual themselves, gemv.hip PRO_RS)
template <int NR>
__global__ void __launch_bounds__(kThreads) car_oneshot_kernel(uint16_t* __restrict__ out,
                                                               const uint16_t* __restrict__ in,
                                                               long n16, Peers peers, int rank,
                                                               uint32_t* epochs, int* err,
                                                               size_t max_bytes, int add_out) {
  __shared__ uint32_t s_e;
  const int b = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) s_e = epochs[b] + 1;
  __syncthreads();
  const uint32_t e = s_e;
  const size_t doff = (size_t)(e & 1) * max_bytes;
  const long per = (n16 + kBlocks - 1) / kBlocks;
  const long lo = min(n16, (long)b * per), hi = min(n16, lo + per);
  const uint4* src = reinterpret_cast<const uint4*>(in);

  // 1. publish my slice
  uint4* mine = reinterpret_cast<uint4*>(peers.data[rank] + doff);
  for (long i = lo + tid; i < hi; i += kThreads) mine[i] = src[i];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: write back dirty L2 lines
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int p = 0; p < NR; ++p) {
      uint32_t* f = reinterpret_cast<uint32_t*>(peers.base[p]) + (size_t)(rank * kBlocks + b) * kFlagStride;
      __hip_atomic_store(f, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  // 2. wait for every peer's slice b
  if (tid < 64) {
    if (tid < NR) {
      const uint32_t* f =
          reinterpret_cast<const uint32_t*>(peers.base[rank]) + (size_t)(tid * kBlocks + b) * kFlagStride;
      long spins = 0;
      while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
        if (++spins > kMaxSpins) {
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: drop stale L1/L2 lines
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();

  // 3. reduce in rank order (bitwise identical on every rank)
  uint4* o = reinterpret_cast<uint4*>(out);
  for (long i = lo + tid; i < hi; i += kThreads) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int p = 0; p < NR; ++p) {
      const uint4 v = p == rank ? src[i] : reinterpret_cast<const uint4*>(peers.data[p] + doff)[i];
      add_bf16x8(acc, v);
    }
    if (add_out) {
      float res[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      add_bf16x8(res, o[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = res[j] + bf2f(f2bf(acc[j]));
    }
    uint4 r;
    r.x = (uint32_t)f2bf(acc[0]) | ((uint32_t)f2bf(acc[1]) << 16);
    r.y = (uint32_t)f2bf(acc[2]) | ((uint32_t)f2bf(acc[3]) << 16);
    r.z = (uint32_t)f2bf(acc[4]) | ((uint32_t)f2bf(acc[5]) << 16);
    r.w = (uint32_t)f2bf(acc[6]) | ((uint32_t)f2bf(acc[7]) << 16);
    o[i] = r;
  }
  if (tid == 0) epochs[b] = e;
}

// Two-shot form for large messages (tensor-parallel prefill chunks; one-shot would read (N-1) x
// the message over the fabric per rank): reduce-scatter then all-gather, each ONE hop over the
// full xGMI mesh, so a rank moves 2 (N-1) / N x the message -- the ring's volume -- but over all
// N-1 links at once and in 2 steps instead of 2 (N-1).
//   data[parity] = | input copy (n16 x 16 B) | reduced (n16 x 16 B, only this rank's slice) |
//   phase 1: block b publishes its piece of the input copy (all slices), flag (rank, b, phase 1)
//            at every peer; then for THIS rank's slice piece b: wait for every peer's phase-1
//            flag b, sum the N copies in rank order (fp32), store bf16 into reduced (own buffer)
//            AND into out; flag (rank, b, phase 2) at every peer;
//   phase 2: for every other slice p: wait for peer p's phase-2 flag b, copy its reduced piece b
//            into out.
// Every rank's result is bitwise the same (the sum of slice p is computed by rank p only).
// In place (out == in) is safe: block b reads every input element it owns (1a, 1b) before it
// writes that element (1b: the same thread, same index; 2: after the phase-1 barriers).
// Phase-2 flags live in the second flag bank (the first is shared with the one-shot kernel: both
// advance the same per-block epochs, so a slot always holds the latest epoch it was raised at).
template <int NR>
__global__ void __launch_bounds__(kThreads) car_twoshot_kernel(uint16_t* __restrict__ out,
                                                               const uint16_t* __restrict__ in, long n16,
                                                               Peers peers, int rank, uint32_t* epochs, int* err,
                                                               size_t max_bytes) {
  __shared__ uint32_t s_e;
  const int b = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) s_e = epochs[b] + 1;
  __syncthreads();
  const uint32_t e = s_e;
  const size_t half = max_bytes / 2;  // input copy | reduced, per parity
  const size_t doff = (size_t)(e & 1) * max_bytes;
  const uint4* src = reinterpret_cast<const uint4*>(in);
  uint4* o = reinterpret_cast<uint4*>(out);
  // slices: rank p owns [p * sl, min(n16, (p + 1) * sl)); block b its piece of every slice
  const long sl = (n16 + NR - 1) / NR;
  const long per = (sl + kBlocks - 1) / kBlocks;
  auto piece = [&](int p, long& lo, long& hi) {
    const long s0 = min(n16, (long)p * sl), s1 = min(n16, s0 + sl);
    lo = min(s1, s0 + (long)b * per);
    hi = min(s1, lo + per);
  };
  auto flag = [&](int owner, int src_rank, int phase) {
    return reinterpret_cast<uint32_t*>(peers.base[owner]) + (size_t)phase * (kFlagBank / 4) +
           (size_t)(src_rank * kBlocks + b) * kFlagStride;
  };
  auto wait = [&](int p, int phase) {
    const uint32_t* f = flag(rank, p, phase);
    long spins = 0;
    while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      if (++spins > kMaxSpins) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  };
  auto signal = [&](int phase) {  // after this block's stores: release, then flag at every peer
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int p = 0; p < NR; ++p) __hip_atomic_store(flag(p, rank, phase), e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  };
  // 1a. publish piece b of every slice of the input
  uint4* mine_in = reinterpret_cast<uint4*>(peers.data[rank] + doff);
#pragma unroll
  for (int p = 0; p < NR; ++p) {
    long lo, hi;
    piece(p, lo, hi);
    for (long i = lo + tid; i < hi; i += kThreads) mine_in[i] = src[i];
  }
  signal(0);
  // 1b. reduce my slice's piece b over the N copies, in rank order
  if (tid < 64) {
    if (tid < NR) wait(tid, 0);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  {
    long lo, hi;
    piece(rank, lo, hi);
    uint4* red = reinterpret_cast<uint4*>(peers.data[rank] + doff + half);
    for (long i = lo + tid; i < hi; i += kThreads) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int p = 0; p < NR; ++p) {
        const uint4 v = p == rank ? src[i] : reinterpret_cast<const uint4*>(peers.data[p] + doff)[i];
        add_bf16x8(acc, v);
      }
      uint4 r;
      r.x = (uint32_t)f2bf(acc[0]) | ((uint32_t)f2bf(acc[1]) << 16);
      r.y = (uint32_t)f2bf(acc[2]) | ((uint32_t)f2bf(acc[3]) << 16);
      r.z = (uint32_t)f2bf(acc[4]) | ((uint32_t)f2bf(acc[5]) << 16);
      r.w = (uint32_t)f2bf(acc[6]) | ((uint32_t)f2bf(acc[7]) << 16);
      red[i] = r;
      o[i] = r;
    }
  }
  signal(1);
  // 2. gather the other ranks' reduced pieces b
  if (tid < 64) {
    if (tid < NR && tid != rank) wait(tid, 1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < NR; ++p) {
    if (p == rank) continue;
    long lo, hi;
    piece(p, lo, hi);
    const uint4* red = reinterpret_cast<const uint4*>(peers.data[p] + doff + half);
    for (long i = lo + tid; i < hi; i += kThreads) o[i] = red[i];
  }
  if (tid == 0) epochs[b] = e;
}

// Broadcast from `root` over the same buffers and per-block epochs (the TP leader's packed step
// metadata: a worker's copy is one hop from the leader's IPC buffer, no host round trip):
//   root: block b publishes its slice into its own buffer (parity e & 1), raises (root, b) at
//         every peer; every other rank waits for (root, b), copies the slice into `out`, raises
//         (rank, b); then EVERY rank waits for every rank's (p, b) >= e before the block ends --
//         nobody starts call e + 2 (the same parity) before everyone finished copying call e.
template <int NR>
__global__ void __launch_bounds__(kThreads) car_bcast_kernel(uint4* __restrict__ out, const uint4* __restrict__ in,
                                                             long n16, Peers peers, int rank, int root,
                                                             uint32_t* epochs, int* err, size_t max_bytes) {
  __shared__ uint32_t s_e;
  const int b = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) s_e = epochs[b] + 1;
  __syncthreads();
  const uint32_t e = s_e;
  const size_t doff = (size_t)(e & 1) * max_bytes;
  const long per = (n16 + kBlocks - 1) / kBlocks;
  const long lo = min(n16, (long)b * per), hi = min(n16, lo + per);
  auto raise_flag = [&]() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int p = 0; p < NR; ++p) {
        uint32_t* f = reinterpret_cast<uint32_t*>(peers.base[p]) + (size_t)(rank * kBlocks + b) * kFlagStride;
        __hip_atomic_store(f, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  };
  auto wait_from = [&](int p) {
    const uint32_t* f = reinterpret_cast<const uint32_t*>(peers.base[rank]) + (size_t)(p * kBlocks + b) * kFlagStride;
    long spins = 0;
    while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      if (++spins > kMaxSpins) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  };
  if (rank == root) {
    uint4* mine = reinterpret_cast<uint4*>(peers.data[rank] + doff);
    for (long i = lo + tid; i < hi; i += kThreads) {
      const uint4 v = in[i];
      mine[i] = v;
      if (out != in) out[i] = v;
    }
    raise_flag();
  } else {
    if (tid == 0) wait_from(root);
    if (tid < 64) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    const uint4* src = reinterpret_cast<const uint4*>(peers.data[root] + doff);
    for (long i = lo + tid; i < hi; i += kThreads) out[i] = src[i];
    raise_flag();
  }
  if (tid < NR) wait_from(tid);  // everyone done with this call's parity
  __syncthreads();
  if (tid == 0) epochs[b] = e;
}

// All-gather (the TP vocab-parallel logits / greedy (max, index) pairs): every rank publishes
// its piece (n4 4-B words) into its own buffer, block b raises (rank, b) at every peer, waits
// for every peer's (p, b) and copies slice b of each piece p into out[p * n4 ...] -- one hop
// per piece, as the one-shot all-reduce, whose flags / parity / epochs it shares.
template <int NR>
__global__ void __launch_bounds__(kThreads) car_allgather_kernel(uint32_t* __restrict__ out,
                                                                 const uint32_t* __restrict__ in, long n4,
                                                                 Peers peers, int rank, uint32_t* epochs,
                                                                 int* err, size_t max_bytes) {
  __shared__ uint32_t s_e;
  const int b = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) s_e = epochs[b] + 1;
  __syncthreads();
  const uint32_t e = s_e;
  const size_t doff = (size_t)(e & 1) * max_bytes;
  const long per = (n4 + kBlocks - 1) / kBlocks;
  const long lo = min(n4, (long)b * per), hi = min(n4, lo + per);
  uint32_t* mine = reinterpret_cast<uint32_t*>(peers.data[rank] + doff);
  for (long i = lo + tid; i < hi; i += kThreads) {
    const uint32_t v = in[i];
    mine[i] = v;
    out[(long)rank * n4 + i] = v;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int p = 0; p < NR; ++p) {
      uint32_t* f = reinterpret_cast<uint32_t*>(peers.base[p]) + (size_t)(rank * kBlocks + b) * kFlagStride;
      __hip_atomic_store(f, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  if (tid < 64) {
    if (tid < NR) {
      const uint32_t* f = reinterpret_cast<const uint32_t*>(peers.base[rank]) + (size_t)(tid * kBlocks + b) * kFlagStride;
      long spins = 0;
      while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
        if (++spins > kMaxSpins) {
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < NR; ++p) {
    if (p == rank) continue;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(peers.data[p] + doff);
    for (long i = lo + tid; i < hi; i += kThreads) out[(long)p * n4 + i] = src[i];
  }
  if (tid == 0) epochs[b] = e;
}

CarState* get(long h) {
  if (h == 0) throw std::runtime_error("custom all-reduce: null handle");
  return reinterpret_cast<CarState*>(h);
}

}  // namespace

long car_create(int rank, int world, long max_bytes, int device, int split) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world)
    throw std::runtime_error("custom all-reduce: bad rank/world");
  if (max_bytes <= 0 || max_bytes % 16) throw std::runtime_error("custom all-reduce: max_bytes % 16");
  auto* s = new CarState;
  s->rank = rank, s->world = world, s->device = device, s->max_bytes = (size_t)max_bytes, s->split = split ? 1 : 0;
  CAR_CHECK(hipSetDevice(device));
  const size_t data_bytes = 2 * (size_t)max_bytes;
  const size_t bytes = kFlagsBytes + (s->split ? 0 : data_bytes);
  if (hipExtMallocWithFlags((void**)&s->buf, bytes, hipDeviceMallocUncached) == hipSuccess) {
    hipIpcMemHandle_t probe;
    if (hipIpcGetMemHandle(&probe, s->buf) == hipSuccess) {
      s->uncached = 1;
    } else {
      (void)hipFree(s->buf);
      s->buf = nullptr;
    }
  }
  (void)hipGetLastError();  // clear a refused uncached allocation / export
  if (!s->buf) CAR_CHECK(hipMalloc(&s->buf, bytes));
  CAR_CHECK(hipMemset(s->buf, 0, kFlagsBytes));
  if (s->split) CAR_CHECK(hipMalloc(&s->dbuf, data_bytes));
  CAR_CHECK(hipMalloc(&s->epochs, kBlocks * sizeof(uint32_t)));
  CAR_CHECK(hipMemset(s->epochs, 0, kBlocks * sizeof(uint32_t)));
  // error word in host-mapped (coherent) memory: the host polls it every engine step with a
  // plain load, no device sync (a wedged or dead peer becomes a Python error, not silent garbage)
  CAR_CHECK(hipHostMalloc(reinterpret_cast<void**>(&s->err_host), sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
  *s->err_host = 0;
  CAR_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&s->err), s->err_host, 0));
  CAR_CHECK(hipDeviceSynchronize());
  s->peers.base[rank] = s->buf;
  s->peers.data[rank] = s->split ? s->dbuf : s->buf + kFlagsBytes;
  return reinterpret_cast<long>(s);
}

// two 64-B handles per rank: the flag buffer, then the data buffer (zeros when not split)
void car_ipc_handle(long h, void* out128) {
  CarState* s = get(h);
  static_assert(sizeof(hipIpcMemHandle_t) == 64, "IPC handle size");
  CAR_CHECK(hipSetDevice(s->device));
  auto* hs = reinterpret_cast<hipIpcMemHandle_t*>(out128);
  CAR_CHECK(hipIpcGetMemHandle(&hs[0], s->buf));
  if (s->split)
    CAR_CHECK(hipIpcGetMemHandle(&hs[1], s->dbuf));
  else
    std::memset(&hs[1], 0, sizeof(hipIpcMemHandle_t));
}

void car_open(long h, const void* handles) {
  CarState* s = get(h);
  CAR_CHECK(hipSetDevice(s->device));
  const auto* hs = reinterpret_cast<const hipIpcMemHandle_t*>(handles);
  for (int p = 0; p < s->world; ++p) {
    if (p == s->rank || s->peers.base[p]) continue;
    void* ptr = nullptr;
    CAR_CHECK(hipIpcOpenMemHandle(&ptr, hs[2 * p], hipIpcMemLazyEnablePeerAccess));
    s->peers.base[p] = reinterpret_cast<uint8_t*>(ptr);
    if (s->split) {
      void* dptr = nullptr;
      CAR_CHECK(hipIpcOpenMemHandle(&dptr, hs[2 * p + 1], hipIpcMemLazyEnablePeerAccess));
      s->peers.data[p] = reinterpret_cast<uint8_t*>(dptr);
    } else {
      s->peers.data[p] = s->peers.base[p] + kFlagsBytes;
    }
  }
}

long car_max_bytes(long h) { return (long)get(h)->max_bytes; }

// bit 0: flags uncached; bit 1: data in its own cached buffer
int car_mem_mode(long h) { return get(h)->uncached | (get(h)->split << 1); }

void car_all_reduce(long h, void* out, const void* in, long numel, hipStream_t st, bool two_shot, bool add_out) {
  CarState* s = get(h);
  if (add_out && (two_shot || out == in)) throw std::runtime_error("custom all-reduce: add form is one-shot, out != in");
  if (numel % 8) throw std::runtime_error("custom all-reduce: numel must be a multiple of 8");
  if ((size_t)numel * 2 * (two_shot ? 2 : 1) > s->max_bytes)
    throw std::runtime_error("custom all-reduce: message too large");
  for (int p = 0; p < s->world; ++p)
    if (!s->peers.base[p]) throw std::runtime_error("custom all-reduce: peers not opened");
  const long n16 = numel / 8;
  dim3 g(kBlocks), blk(kThreads);
  auto* o = static_cast<uint16_t*>(out);
  auto* i = static_cast<const uint16_t*>(in);
  if (two_shot) {
    switch (s->world) {
      case 1: car_twoshot_kernel<1><<<g, blk, 0, st>>>(o, i, n16, s->peers, s->rank, s->epochs, s->err, s->max_bytes); break;
      case 2: car_twoshot_kernel<2><<<g, blk, 0, st>>>(o, i, n16, s->peers, s->rank, s->epochs, s->err, s->max_bytes); break;
      case 4: car_twoshot_kernel<4><<<g, blk, 0, st>>>(o, i, n16, s->peers, s->rank, s->epochs, s->err, s->max_bytes); break;
      case 8: car_twoshot_kernel<8><<<g, blk, 0, st>>>(o, i, n16, s->peers, s->rank, s->epochs, s->err, s->max_bytes); break;
      default: throw std::runtime_error("custom all-reduce: world must be 1, 2, 4 or 8");
    }
    CAR_CHECK(hipGetLastError());
    return;
  }
  switch (s->world) {
    case 1: car_oneshot_kernel<1><<<g, blk, 0, st>>>(o, i, n16, s->peers, s->rank, s->epochs, s->err, s->max_bytes, add_out); break;
    case 2: car_oneshot_kernel<2><<<g, blk, 0, st>>>(o, i, n16, s->peers, s->rank, s->epochs, s->err, s->max_bytes, add_out); break;
    case 4: car_oneshot_kernel<4><<<g, blk, 0, st>>>(o, i, n16, s->peers, s->rank, s->epochs, s->err, s->max_bytes, add_out); break;
    case 8: car_oneshot_kernel<8><<<g, blk, 0, st>>>(o, i, n16, s->peers, s->rank, s->epochs, s->err, s->max_bytes, add_out); break;
    default: throw std::runtime_error("custom all-reduce: world must be 1, 2, 4 or 8");
  }
  CAR_CHECK(hipGetLastError());
}

void car_broadcast(long h, void* out, const void* in, long nbytes, int root, hipStream_t st) {
  CarState* s = get(h);
  if (nbytes % 16) throw std::runtime_error("custom broadcast: bytes must be a multiple of 16");
  if ((size_t)nbytes > s->max_bytes) throw std::runtime_error("custom broadcast: message too large");
  if (root < 0 || root >= s->world) throw std::runtime_error("custom broadcast: bad root");
  for (int p = 0; p < s->world; ++p)
    if (!s->peers.base[p]) throw std::runtime_error("custom broadcast: peers not opened");
  const long n16 = nbytes / 16;
  auto* o = static_cast<uint4*>(out);
  auto* i = static_cast<const uint4*>(in);
  dim3 g(kBlocks), blk(kThreads);
  switch (s->world) {
    case 1: car_bcast_kernel<1><<<g, blk, 0, st>>>(o, i, n16, s->peers, s->rank, root, s->epochs, s->err, s->max_bytes); break;
    case 2: car_bcast_kernel<2><<<g, blk, 0, st>>>(o, i, n16, s->peers, s->rank, root, s->epochs, s->err, s->max_bytes); break;
    case 4: car_bcast_kernel<4><<<g, blk, 0, st>>>(o, i, n16, s->peers, s->rank, root, s->epochs, s->err, s->max_bytes); break;
    case 8: car_bcast_kernel<8><<<g, blk, 0, st>>>(o, i, n16, s->peers, s->rank, root, s->epochs, s->err, s->max_bytes); break;
    default: throw std::runtime_error("custom broadcast: world must be 1, 2, 4 or 8");
  }
  CAR_CHECK(hipGetLastError());
}

void car_all_gather(long h, void* out, long out_bytes, const void* in, long nbytes, hipStream_t st) {
  CarState* s = get(h);
  if (nbytes % 4) throw std::runtime_error("custom all-gather: bytes must be a multiple of 4");
  if (out_bytes != nbytes * (long)s->world) throw std::runtime_error("custom all-gather: out must be world x piece");
  if ((size_t)nbytes > s->max_bytes) throw std::runtime_error("custom all-gather: piece too large");
  for (int p = 0; p < s->world; ++p)
    if (!s->peers.base[p]) throw std::runtime_error("custom all-gather: peers not opened");
  const long n4 = nbytes / 4;
  auto* o = static_cast<uint32_t*>(out);
  auto* i = static_cast<const uint32_t*>(in);
  dim3 g(kBlocks), blk(kThreads);
  switch (s->world) {
    case 1: car_allgather_kernel<1><<<g, blk, 0, st>>>(o, i, n4, s->peers, s->rank, s->epochs, s->err, s->max_bytes); break;
    case 2: car_allgather_kernel<2><<<g, blk, 0, st>>>(o, i, n4, s->peers, s->rank, s->epochs, s->err, s->max_bytes); break;
    case 4: car_allgather_kernel<4><<<g, blk, 0, st>>>(o, i, n4, s->peers, s->rank, s->epochs, s->err, s->max_bytes); break;
    case 8: car_allgather_kernel<8><<<g, blk, 0, st>>>(o, i, n4, s->peers, s->rank, s->epochs, s->err, s->max_bytes); break;
    default: throw std::runtime_error("custom all-gather: world must be 1, 2, 4 or 8");
  }
  CAR_CHECK(hipGetLastError());
}

int car_error(long h) {
  CarState* s = get(h);
  return __atomic_load_n(s->err_host, __ATOMIC_ACQUIRE);
}

void car_destroy(long h) {
  CarState* s = get(h);
  hipSetDevice(s->device);
  hipDeviceSynchronize();
  for (int p = 0; p < s->world; ++p)
    if (p != s->rank && s->peers.base[p]) {
      hipIpcCloseMemHandle(s->peers.base[p]);
      if (s->split && s->peers.data[p]) hipIpcCloseMemHandle(s->peers.data[p]);
    }
  hipFree(s->buf);
  if (s->dbuf) hipFree(s->dbuf);
  hipFree(s->epochs);
  hipHostFree(s->err_host);
  delete s;
}

}  // namespace mlop
