// Lazily backed device arenas for the paged KV cache (HIP virtual memory management).
//
// Why: a predictor's KV pool is most of the 288 GB of HBM (134 GB for the default
// Llama-3-8B bench), and hipMalloc of that much memory right after another process freed
// it waits for the driver to scrub the pages: 0.7-4.8 s measured (scripts/run66.sh,
// profiles/r02_kv_lazy_map.md) on top of a 0.6 s start-up.  That wait sits on the
// CR -> ready path of every deploy, canary and crash-restart.  Instead the engine reserves
// the whole virtual range at once (no physical memory), backs + zeroes the first chunk of
// pages synchronously, reports ready, and a native worker thread backs the remaining
// chunks (hipMemCreate + hipMemMap + hipMemSetAccess, zeroed on its own stream) while the
// engine serves; the block allocator only ever hands out pages of completed chunks
// (runtime/kv_cache.py), so no kernel touches an unbacked address.
//
// Layout: n_regions regions of `region_stride` bytes (one per K / V layer tensor); chunk c
// backs bytes [c * chunk_bytes, (c + 1) * chunk_bytes) of EVERY region, so a page id is
// usable in every layer as soon as its chunk completes.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace mlop {

namespace {

struct Arena {
  int device = 0;
  char* base = nullptr;
  size_t reserved = 0;
  std::mutex mu;  // guards maps
  std::vector<std::pair<size_t, std::pair<size_t, hipMemGenericAllocationHandle_t>>> maps;
  std::atomic<long> chunks_ready{0};
  std::atomic<int> error{0};
  std::atomic<bool> stop{false};
  std::thread worker;

  ~Arena() {
    stop = true;
    if (worker.joinable()) worker.join();
    (void)hipSetDevice(device);
    (void)hipDeviceSynchronize();
    for (auto& m : maps) {
      (void)hipMemUnmap(base + m.first, m.second.first);
      (void)hipMemRelease(m.second.second);
    }
    if (base) (void)hipMemAddressFree(base, reserved);
  }
};

std::mutex g_mu;
std::map<uintptr_t, std::weak_ptr<Arena>> g_arenas;  // base address -> arena

hipMemAllocationProp device_prop(int device) {
  hipMemAllocationProp prop{};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = device;
  return prop;
}

std::shared_ptr<Arena> find(const void* base) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_arenas.find(reinterpret_cast<uintptr_t>(base));
  return it == g_arenas.end() ? nullptr : it->second.lock();
}

// back [off, off + bytes) with fresh physical memory, device read/write
hipError_t map_range(Arena& a, size_t off, size_t bytes) {
  hipMemAllocationProp prop = device_prop(a.device);
  hipMemGenericAllocationHandle_t h;
  hipError_t e = hipMemCreate(&h, bytes, &prop, 0);
  if (e != hipSuccess) return e;
  e = hipMemMap(a.base + off, bytes, 0, h, 0);
  if (e != hipSuccess) {
    (void)hipMemRelease(h);
    return e;
  }
  hipMemAccessDesc acc{};
  acc.location.type = hipMemLocationTypeDevice;
  acc.location.id = a.device;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  e = hipMemSetAccess(a.base + off, bytes, &acc, 1);
  std::lock_guard<std::mutex> g(a.mu);
  a.maps.push_back({off, {bytes, h}});
  return e;
}

// back + zero chunk c of every region; zeroing runs on `st` and is waited for before return
hipError_t map_chunk(Arena& a, long c, size_t region_stride, int n_regions, size_t chunk_bytes,
                     hipStream_t st) {
  for (int r = 0; r < n_regions; ++r) {
    const size_t off = (size_t)r * region_stride + (size_t)c * chunk_bytes;
    hipError_t e = map_range(a, off, chunk_bytes);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(a.base + off, 0, chunk_bytes, st);
    if (e != hipSuccess) return e;
  }
  return hipStreamSynchronize(st);
}

}  // namespace

bool vmm_supported(int device) {
  int v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeVirtualMemoryManagementSupported, device) != hipSuccess)
    return false;
  return v != 0;
}

long vmm_granularity(int device) {
  hipMemAllocationProp prop = device_prop(device);
  size_t g = 0;
  if (hipMemGetAllocationGranularity(&g, &prop, hipMemAllocationGranularityMinimum) != hipSuccess) return -1;
  return (long)g;
}

// Reserve `bytes` of device virtual address space (rounded up to the granularity).  The
// returned shared_ptr owns the arena; the caller ties it to the tensor storage over `base`.
std::shared_ptr<void> vmm_reserve(long bytes, int device, void** base_out, long* reserved_out) {
  const long g = vmm_granularity(device);
  if (g <= 0) return nullptr;
  auto a = std::make_shared<Arena>();
  a->device = device;
  a->reserved = (size_t)((bytes + g - 1) / g * g);
  (void)hipSetDevice(device);
  void* p = nullptr;
  if (hipMemAddressReserve(&p, a->reserved, (size_t)g, nullptr, 0) != hipSuccess) return nullptr;
  a->base = (char*)p;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    g_arenas[reinterpret_cast<uintptr_t>(p)] = a;
  }
  *base_out = p;
  *reserved_out = (long)a->reserved;
  return std::shared_ptr<void>(a, a.get());
}

void vmm_forget(void* base) {
  std::lock_guard<std::mutex> g(g_mu);
  g_arenas.erase(reinterpret_cast<uintptr_t>(base));
}

// Back + zero chunks [first, first + count) of every region.  Synchronous unless `async`:
// then a native worker thread does it chunk by chunk (its own non-blocking stream), and
// vmm_chunks_ready() reports progress.  Returns false on an immediate error.
bool vmm_map_chunks(void* base, long region_stride, int n_regions, long chunk_bytes, long first, long count,
                    bool async) {
  auto a = find(base);
  if (!a) return false;
  const long g = vmm_granularity(a->device);
  if (g <= 0 || region_stride % g || chunk_bytes % g ||
      (size_t)region_stride * n_regions > a->reserved || (first + count) * chunk_bytes > region_stride)
    return false;
  if (!async) {
    (void)hipSetDevice(a->device);
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return false;
    bool ok = true;
    for (long c = first; c < first + count && ok; ++c) {
      ok = map_chunk(*a, c, (size_t)region_stride, n_regions, (size_t)chunk_bytes, st) == hipSuccess;
      if (ok) a->chunks_ready.store(c + 1);
    }
    (void)hipStreamDestroy(st);
    if (!ok) a->error = 1;
    return ok;
  }
  if (a->worker.joinable()) return false;  // one background fill per arena
  Arena* ap = a.get();  // the arena's destructor joins the worker before anything is freed
  a->worker = std::thread([ap, region_stride, n_regions, chunk_bytes, first, count] {
    (void)hipSetDevice(ap->device);
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
      ap->error = 1;
      return;
    }
    for (long c = first; c < first + count && !ap->stop.load(); ++c) {
      if (map_chunk(*ap, c, (size_t)region_stride, n_regions, (size_t)chunk_bytes, st) != hipSuccess) {
        ap->error = 1;
        break;
      }
      ap->chunks_ready.store(c + 1);
    }
    (void)hipStreamDestroy(st);
  });
  return true;
}

long vmm_chunks_ready(void* base) {
  auto a = find(base);
  return a ? a->chunks_ready.load() : -1;
}

int vmm_error(void* base) {
  auto a = find(base);
  return a ? a->error.load() : 1;
}

}  // namespace mlop
