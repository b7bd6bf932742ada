// Expert-parallel MoE dispatch / combine over xGMI peer memory (config 5: DP attention + EP).
//
// Every rank holds its own tokens; each MoE layer sends every routed (token, expert) slot to the
// rank that owns the expert and brings the expert output back.  RCCL's all_to_all needs the
// per-peer counts on the host (a sync) or a fixed worst-case split (each rank then ships P x its
// routed rows, the old path in parallel/moe.py).  Here the exchange is device-side and EXACT:
// only routed rows cross the fabric, and nothing waits on the host, so it is captured into the
// decode hipGraphs like the K15 all-reduce (allreduce.hip, whose flag protocol this reuses).
//
// Per rank one IPC-exported UNCACHED buffer (peers write into it; see allreduce.hip "Memory"):
//   flags [3 phases][P sources] (64-B lines) | table [P][E] int32 | recv [P*tcap*k][H] bf16 |
//   meta [P*tcap*k] int32 | back [tcap*k][H] bf16
// and per MoE layer (epoch e = one more than the last, kept on the device):
//   1. ep_count_kernel (n_slots/1024 workgroups): per-(workgroup, expert) counts of this rank's
//      T*k slots and each slot's rank inside its (workgroup, expert) segment -- wave ballots, so
//      the row order is the slot order (deterministic);
//   2. ep_plan_kernel (1 workgroup, small arrays only): this rank's per-expert counts go into
//      EVERY peer's table row [rank] + a phase-0 flag; once all P rows are in, every rank knows
//      the whole [P][E] count matrix, so the destination row of every slot is fixed without a
//      second round trip: at the owner d of expert x the received rows are grouped by expert
//      (x's segment starts after d's lower experts' totals) and, inside x's segment, by source
//      rank.  Also this rank's own received layout: offsets of its local experts (the grouped
//      GEMM's) and the received row count;
//   3. ep_dispatch_kernel (one wave per slot): row x[t] -> the owner's recv at its final row,
//      (source, slot) -> meta; the last workgroup to finish (ticket) raises the phase-1 flag of
//      every peer;
//   4. ep_recv_kernel (<= 64 workgroups): wait for all P phase-1 flags, copy the received rows
//      out of the uncached buffer into the (cached) grouped GEMM input, meta beside them;
//      -> grouped GEMMs (gemm.hip, K13) over the local experts with the device offsets;
//   5. ep_combine_send_kernel: expert output row i -> its source's back[slot]; ticket -> phase-2
//      flags;
//   6. ep_combine_kernel (<= 64 workgroups): wait for all P phase-2 flags, out[t] = sum_j
//      topw[t, j] * back[t*k + j] (fp32, one bf16 rounding; rank-independent order).
// One buffer suffices per phase: a rank issues layer n+1's dispatch only after its layer-n
// combine saw every peer's phase-2 flag, which each peer raises after it finished reading its
// recv / table of layer n.  Grids that spin are capped at 64 workgroups (two ranks may share one
// GPU in the tests) and every spin is bounded (error word, never a hang).
#include "common.h"
#include "launch.h"

#include <stdexcept>
#include <string>

namespace mlop {

namespace {

constexpr int kEpMaxRanks = 8;
constexpr int kEpMaxE = 64;
constexpr int kEpCountThreads = 1024;  // slots per count workgroup
constexpr int kEpMaxCountWg = 64;      // n_slots <= 65536
constexpr int kEpSpinWg = 64;          // workgroups of the kernels that wait on peers
constexpr int kEpCopyWg = 256;         // workgroups of the kernels that only write
constexpr int kFlagLine = 16;          // u32 per flag: one 64-B line
constexpr long kEpMaxSpins = 1L << 26;

struct EpPeers {
  uint8_t* base[kEpMaxRanks];
};

struct EpState {
  int rank = 0, world = 1, device = 0, E = 0, n_local = 0, k = 0, H = 0, tcap = 0;
  int uncached = 0;
  size_t off_table = 0, off_recv = 0, off_meta = 0, off_back = 0, bytes = 0;
  uint8_t* buf = nullptr;  // IPC-exported
  EpPeers peers{};
  uint32_t* epoch = nullptr;  // [1]
  int* tickets = nullptr;     // [2]
  int* err = nullptr;         // [1] device alias of err_host (host-mapped, polled without a sync)
  int* err_host = nullptr;
  int* wcnt = nullptr;        // [kEpMaxCountWg][E]
  int* wbase = nullptr;       // [kEpMaxCountWg][E]
  int* lrank = nullptr;       // [tcap * k]
  int* info = nullptr;        // [n_local + 1]: local expert offsets in the received rows
  int* meta_l = nullptr;      // [P * tcap * k]
};

#define EP_CHECK(x)                                                                                 \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess)                                                                           \
      throw std::runtime_error(std::string("ep exchange: ") + #x + ": " + hipGetErrorString(e_));   \
  } while (0)

__device__ __forceinline__ uint32_t* flag_at(uint8_t* base, int phase, int src) {
  return reinterpret_cast<uint32_t*>(base) + (size_t)(phase * kEpMaxRanks + src) * kFlagLine;
}

// lanes 0..P-1 of wave 0 wait until the phase flag of every source reached epoch e, then a
// system-scope acquire; the whole workgroup passes the barrier after
__device__ __forceinline__ void wait_flags(uint8_t* mine, int phase, int P, uint32_t e, int* err) {
  if (threadIdx.x < 64) {
    if ((int)threadIdx.x < P) {
      const uint32_t* f = flag_at(mine, phase, threadIdx.x);
      long spins = 0;
      while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
        if (++spins > kEpMaxSpins) {
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
}

// every workgroup: its stores complete, a system release, a ticket; the last one raises `phase`
// for this rank at every peer
__device__ __forceinline__ void ticket_and_signal(EpPeers peers, int P, int rank, int phase, uint32_t e,
                                                  int* ticket) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int tk = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (tk == (int)gridDim.x - 1) {
      __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      for (int p = 0; p < P; ++p)
        __hip_atomic_store(flag_at(peers.base[p], phase, rank), e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// 1. per-(workgroup, expert) counts and ranks, slot order
__global__ void __launch_bounds__(kEpCountThreads) ep_count_kernel(int* __restrict__ wcnt, int* __restrict__ lrank,
                                                                  const int* __restrict__ topi, int n_slots, int E) {
  __shared__ int wc[kEpCountThreads / 64][kEpMaxE];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int s = blockIdx.x * kEpCountThreads + threadIdx.x;
  const int e = s < n_slots ? topi[s] : -1;
  const unsigned long long lt = (1ull << lane) - 1ull;
  int r = 0;
  for (int x = 0; x < E; ++x) {
    const unsigned long long m = __ballot(e == x);
    if (e == x) r = __popcll(m & lt);
    if (lane == 0) wc[wv][x] = __popcll(m);
  }
  __syncthreads();
  if ((int)threadIdx.x < E) {
    const int x = threadIdx.x;
    int acc = 0;
    for (int w = 0; w < kEpCountThreads / 64; ++w) {
      const int c = wc[w][x];
      wc[w][x] = acc;
      acc += c;
    }
    wcnt[blockIdx.x * E + x] = acc;
  }
  __syncthreads();
  if (s < n_slots) lrank[s] = (e >= 0 && e < E) ? wc[wv][e] + r : -1;
}

// 2. counts exchange + destination rows + this rank's received layout (one workgroup)
__global__ void __launch_bounds__(256) ep_plan_kernel(EpPeers peers, int P, int rank, int E, int n_local, int G,
                                                     uint32_t* epoch, int* err, const int* __restrict__ wcnt,
                                                     int* __restrict__ wbase, int* __restrict__ info,
                                                     int* __restrict__ offsets_out, size_t off_table) {
  __shared__ int mine[kEpMaxE];
  __shared__ int tab[kEpMaxRanks][kEpMaxE];
  __shared__ uint32_t s_e;
  const int tid = threadIdx.x;
  if (tid == 0) {
    s_e = epoch[0] + 1;
    epoch[0] = s_e;  // every later kernel of this layer reads it
  }
  if (tid < E) {
    int c = 0;
    for (int g = 0; g < G; ++g) c += wcnt[g * E + tid];
    mine[tid] = c;
  }
  __syncthreads();
  const uint32_t e = s_e;
  for (int i = tid; i < P * E; i += blockDim.x) {  // my row of every peer's table
    const int p = i / E, x = i % E;
    reinterpret_cast<int*>(peers.base[p] + off_table)[rank * E + x] = mine[x];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int p = 0; p < P; ++p)
      __hip_atomic_store(flag_at(peers.base[p], 0, rank), e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  wait_flags(peers.base[rank], 0, P, e, err);
  for (int i = tid; i < P * E; i += blockDim.x)
    tab[i / E][i % E] = __hip_atomic_load(reinterpret_cast<const int*>(peers.base[rank] + off_table) + i,
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __syncthreads();
  if (tid < E) {
    const int x = tid, d0 = (x / n_local) * n_local;
    int start = 0;
    for (int x2 = d0; x2 < x; ++x2)
      for (int s = 0; s < P; ++s) start += tab[s][x2];
    for (int s = 0; s < rank; ++s) start += tab[s][x];
    for (int g = 0; g < G; ++g) {  // segments of my count workgroups, in order
      wbase[g * E + x] = start;
      start += wcnt[g * E + x];
    }
  }
  if (tid == 0) {
    int acc = 0;
    for (int j = 0; j < n_local; ++j) {
      info[j] = acc;
      offsets_out[j] = acc;
      for (int s = 0; s < P; ++s) acc += tab[s][rank * n_local + j];
    }
    info[n_local] = acc;
    offsets_out[n_local] = acc;
  }
}

// 3. rows to their owners (one wave per slot)
__global__ void __launch_bounds__(256) ep_dispatch_kernel(EpPeers peers, int P, int rank, int E, int n_local, int k,
                                                         int H, int n_slots, const uint16_t* __restrict__ x,
                                                         const int* __restrict__ topi,
                                                         const int* __restrict__ wbase,
                                                         const int* __restrict__ lrank, const uint32_t* epoch,
                                                         int* ticket, size_t off_recv, size_t off_meta) {
  const int lane = threadIdx.x & 63;
  const int waves = gridDim.x * (blockDim.x >> 6);
  const int n16 = H / 8;
  for (int s = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); s < n_slots; s += waves) {
    const int ex = topi[s];
    if (ex < 0 || ex >= E) continue;
    const int d = ex / n_local;
    const int row = wbase[(s / kEpCountThreads) * E + ex] + lrank[s];
    const u32x4* src = reinterpret_cast<const u32x4*>(x + (size_t)(s / k) * H);
    u32x4* dst = reinterpret_cast<u32x4*>(peers.base[d] + off_recv + (size_t)row * H * 2);
    for (int c = lane; c < n16; c += 64) dst[c] = src[c];
    if (lane == 0) reinterpret_cast<int*>(peers.base[d] + off_meta)[row] = (rank << 24) | s;
  }
  ticket_and_signal(peers, P, rank, 1, epoch[0], ticket);
}

// 4. received rows -> the grouped GEMM's input (cached memory)
__global__ void __launch_bounds__(256) ep_recv_kernel(uint16_t* __restrict__ xp, int* __restrict__ meta_l,
                                                     long xp_rows, EpPeers peers, int P, int rank, int n_local,
                                                     int H, const uint32_t* epoch, int* err,
                                                     const int* __restrict__ info, size_t off_recv,
                                                     size_t off_meta) {
  wait_flags(peers.base[rank], 1, P, epoch[0], err);
  long n = info[n_local];
  if (n > xp_rows) {  // a peer sent more than the agreed capacity: never write past xp
    if (threadIdx.x == 0) __hip_atomic_store(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    n = xp_rows;
  }
  const long n16 = (long)H / 8;
  const u32x4* src = reinterpret_cast<const u32x4*>(peers.base[rank] + off_recv);
  u32x4* dst = reinterpret_cast<u32x4*>(xp);
  const long total = n * n16;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x)
    dst[i] = src[i];
  const int* meta = reinterpret_cast<const int*>(peers.base[rank] + off_meta);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    meta_l[i] = meta[i];
}

// 5. expert outputs back to their sources (one wave per row)
__global__ void __launch_bounds__(256) ep_combine_send_kernel(EpPeers peers, int P, int rank, int n_local, int H,
                                                             long y_rows, const uint16_t* __restrict__ y,
                                                             const int* __restrict__ meta_l,
                                                             const int* __restrict__ info, const uint32_t* epoch,
                                                             int* ticket, size_t off_back) {
  const int lane = threadIdx.x & 63;
  const long waves = (long)gridDim.x * (blockDim.x >> 6);
  long n = info[n_local];
  if (n > y_rows) n = y_rows;
  const int n16 = H / 8;
  for (long i = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < n; i += waves) {
    const int m = meta_l[i];
    const int s = (m >> 24) & 0xff, slot = m & 0xffffff;
    if (s >= P) continue;
    const u32x4* src = reinterpret_cast<const u32x4*>(y + (size_t)i * H);
    u32x4* dst = reinterpret_cast<u32x4*>(peers.base[s] + off_back + (size_t)slot * H * 2);
    for (int c = lane; c < n16; c += 64) dst[c] = src[c];
  }
  ticket_and_signal(peers, P, rank, 2, epoch[0], ticket);
}

// 6. weighted sum of each token's k expert outputs
__global__ void __launch_bounds__(256) ep_combine_kernel(uint16_t* __restrict__ out, const float* __restrict__ topw,
                                                        const int* __restrict__ topi, int T, int k, int H, int E,
                                                        EpPeers peers, int P, int rank, const uint32_t* epoch,
                                                        int* err, size_t off_back) {
  wait_flags(peers.base[rank], 2, P, epoch[0], err);
  const uint16_t* back = reinterpret_cast<const uint16_t*>(peers.base[rank] + off_back);
  const int n8 = H / 8;
  const long total = (long)T * n8;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int t = (int)(i / n8), c = (int)(i % n8) * 8;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < k; ++j) {
      const int ex = topi[t * k + j];
      if (ex < 0 || ex >= E) continue;
      const float w = topw[t * k + j];
      const u32x4 v = *reinterpret_cast<const u32x4*>(back + ((size_t)(t * k + j) * H + c));
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

EpState* ep_get(long h) {
  if (h == 0) throw std::runtime_error("ep exchange: null handle");
  return reinterpret_cast<EpState*>(h);
}

void ep_ready(EpState* s) {
  for (int p = 0; p < s->world; ++p)
    if (!s->peers.base[p]) throw std::runtime_error("ep exchange: peers not opened");
}

}  // namespace

long ep_create(int rank, int world, int E, int k, int H, int tcap, int device) {
  if (world < 1 || world > kEpMaxRanks || rank < 0 || rank >= world) throw std::runtime_error("ep exchange: bad rank/world");
  if (E < 1 || E > kEpMaxE || E % world) throw std::runtime_error("ep exchange: experts must divide by ranks (<= 64)");
  if (H % 8 || k < 1 || tcap < 1 || (long)tcap * k > (long)kEpMaxCountWg * kEpCountThreads)
    throw std::runtime_error("ep exchange: H % 8, k >= 1, tcap * k <= 65536");
  auto* s = new EpState;
  s->rank = rank, s->world = world, s->device = device, s->E = E, s->n_local = E / world, s->k = k, s->H = H;
  s->tcap = tcap;
  const size_t rows_in = (size_t)world * tcap * k, rows_out = (size_t)tcap * k;
  auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
  s->off_table = al((size_t)3 * kEpMaxRanks * kFlagLine * 4);
  s->off_recv = al(s->off_table + (size_t)kEpMaxRanks * kEpMaxE * 4);
  s->off_meta = al(s->off_recv + rows_in * H * 2);
  s->off_back = al(s->off_meta + rows_in * 4);
  s->bytes = al(s->off_back + rows_out * H * 2);
  EP_CHECK(hipSetDevice(device));
  if (hipExtMallocWithFlags((void**)&s->buf, s->bytes, hipDeviceMallocUncached) == hipSuccess) {
    hipIpcMemHandle_t probe;
    if (hipIpcGetMemHandle(&probe, s->buf) == hipSuccess) {
      s->uncached = 1;
    } else {
      (void)hipFree(s->buf);
      s->buf = nullptr;
    }
  }
  (void)hipGetLastError();
  if (!s->buf) EP_CHECK(hipMalloc(&s->buf, s->bytes));
  EP_CHECK(hipMemset(s->buf, 0, s->off_recv));  // flags + table
  EP_CHECK(hipMalloc(&s->epoch, sizeof(uint32_t)));
  EP_CHECK(hipMemset(s->epoch, 0, sizeof(uint32_t)));
  EP_CHECK(hipMalloc(&s->tickets, 2 * sizeof(int)));
  EP_CHECK(hipMemset(s->tickets, 0, 2 * sizeof(int)));
  EP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&s->err_host), sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
  *s->err_host = 0;
  EP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&s->err), s->err_host, 0));
  EP_CHECK(hipMalloc(&s->wcnt, (size_t)kEpMaxCountWg * E * sizeof(int)));
  EP_CHECK(hipMalloc(&s->wbase, (size_t)kEpMaxCountWg * E * sizeof(int)));
  EP_CHECK(hipMalloc(&s->lrank, rows_out * sizeof(int)));
  EP_CHECK(hipMalloc(&s->info, (size_t)(s->n_local + 1) * sizeof(int)));
  EP_CHECK(hipMalloc(&s->meta_l, rows_in * sizeof(int)));
  EP_CHECK(hipDeviceSynchronize());
  s->peers.base[rank] = s->buf;
  return reinterpret_cast<long>(s);
}

void ep_ipc_handle(long h, void* out64) {
  EpState* s = ep_get(h);
  EP_CHECK(hipSetDevice(s->device));
  EP_CHECK(hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(out64), s->buf));
}

void ep_open(long h, const void* handles) {
  EpState* s = ep_get(h);
  EP_CHECK(hipSetDevice(s->device));
  const auto* hs = reinterpret_cast<const hipIpcMemHandle_t*>(handles);
  for (int p = 0; p < s->world; ++p) {
    if (p == s->rank || s->peers.base[p]) continue;
    void* ptr = nullptr;
    EP_CHECK(hipIpcOpenMemHandle(&ptr, hs[p], hipIpcMemLazyEnablePeerAccess));
    s->peers.base[p] = reinterpret_cast<uint8_t*>(ptr);
  }
}

int ep_mem_mode(long h) { return ep_get(h)->uncached; }

int ep_world(long h) { return ep_get(h)->world; }
int ep_local_experts(long h) { return ep_get(h)->n_local; }
int ep_hidden(long h) { return ep_get(h)->H; }
int ep_topk(long h) { return ep_get(h)->k; }
int ep_tcap(long h) { return ep_get(h)->tcap; }

void ep_dispatch(long h, void* xp, long xp_rows, int* offsets, const void* x, const int* topi, int T, hipStream_t st) {
  EpState* s = ep_get(h);
  ep_ready(s);
  if (T > s->tcap) throw std::runtime_error("ep exchange: T exceeds the buffer capacity");
  const int n_slots = T * s->k;
  const int G = std::max(1, cdiv(n_slots, kEpCountThreads));
  ep_count_kernel<<<G, kEpCountThreads, 0, st>>>(s->wcnt, s->lrank, topi, n_slots, s->E);
  ep_plan_kernel<<<1, 256, 0, st>>>(s->peers, s->world, s->rank, s->E, s->n_local, G, s->epoch, s->err, s->wcnt,
                                    s->wbase, s->info, offsets, s->off_table);
  const int gd = std::max(1, std::min(kEpCopyWg, cdiv(n_slots, 4)));
  ep_dispatch_kernel<<<gd, 256, 0, st>>>(s->peers, s->world, s->rank, s->E, s->n_local, s->k, s->H, n_slots,
                                         (const uint16_t*)x, topi, s->wbase, s->lrank, s->epoch, s->tickets,
                                         s->off_recv, s->off_meta);
  ep_recv_kernel<<<kEpSpinWg, 256, 0, st>>>((uint16_t*)xp, s->meta_l, xp_rows, s->peers, s->world, s->rank,
                                            s->n_local, s->H, s->epoch, s->err, s->info, s->off_recv, s->off_meta);
  EP_CHECK(hipGetLastError());
}

void ep_combine(long h, void* out, const void* y, long y_rows, const float* topw, const int* topi, int T,
                hipStream_t st) {
  EpState* s = ep_get(h);
  ep_ready(s);
  const int gs = std::max(1, std::min(kEpCopyWg, (int)std::min<long>(y_rows / 4 + 1, 1 << 20)));
  ep_combine_send_kernel<<<gs, 256, 0, st>>>(s->peers, s->world, s->rank, s->n_local, s->H, y_rows,
                                             (const uint16_t*)y, s->meta_l, s->info, s->epoch, s->tickets + 1,
                                             s->off_back);
  ep_combine_kernel<<<kEpSpinWg, 256, 0, st>>>((uint16_t*)out, topw, topi, T, s->k, s->H, s->E, s->peers,
                                               s->world, s->rank, s->epoch, s->err, s->off_back);
  EP_CHECK(hipGetLastError());
}

int ep_error(long h) {
  EpState* s = ep_get(h);
  return __atomic_load_n(s->err_host, __ATOMIC_ACQUIRE);
}

void ep_destroy(long h) {
  EpState* s = ep_get(h);
  hipSetDevice(s->device);
  hipDeviceSynchronize();
  for (int p = 0; p < s->world; ++p)
    if (p != s->rank && s->peers.base[p]) hipIpcCloseMemHandle(s->peers.base[p]);
  hipFree(s->buf);
  for (void* q : {(void*)s->epoch, (void*)s->tickets, (void*)s->wcnt, (void*)s->wbase, (void*)s->lrank,
                  (void*)s->info, (void*)s->meta_l})
    hipFree(q);
  hipHostFree(s->err_host);
  delete s;
}

}  // namespace mlop
