// Host-side race / memory screen of the lazily backed KV arena (ops/csrc/vmm.hip).
//
// vmm.hip is the runtime's one piece of multi-threaded native host code: a worker thread
// backs + zeroes chunks of a reserved virtual range while the serving thread polls
// vmm_chunks_ready(), looks arenas up in a global map, and may drop the arena (its
// destructor stops and joins the worker) at any time.  This harness drives exactly those
// interleavings from several threads and is built twice (+ a plain build) by scripts/build_sanitized.sh:
//   * ThreadSanitizer  (-Xarch_host -fsanitize=thread)              data races, lock order
//   * AddressSanitizer + UBSan (-Xarch_host -fsanitize=address,undefined)   use-after-free of
//     the arena / map entries, leaks, UB in the offset arithmetic
// Sanitizers instrument the host code only (the pool runs no GPU ASan / XNACK); the GPU
// work (hipMemsetAsync zero fill, a check kernel) runs uninstrumented.  Run on the GPU box
// by tests/test_native_sanitizers_gpu.py.  Exit 0 = every scenario passed and the
// sanitizer reported nothing (both runtimes exit non-zero on a report).
#include "../../mlopamd/ops/csrc/vmm.hip"

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

using namespace mlop;

#define CHECK(c)                                                               \
  do {                                                                         \
    if (!(c)) {                                                                \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(2);                                                            \
    }                                                                          \
  } while (0)

// counts non-zero bytes of a backed chunk (the worker must have zeroed it)
__global__ void count_nonzero(const unsigned* p, size_t n, unsigned* out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned c = 0;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) c += p[i] != 0u;
  if (c) atomicAdd(out, c);
}

// poll progress from `threads` threads until `target` chunks are ready; progress must be
// monotonic and the error flag clear
static void poll_until(void* base, long target, int threads) {
  std::vector<std::thread> ts;
  std::atomic<bool> fail{false};
  for (int t = 0; t < threads; ++t)
    ts.emplace_back([&] {
      long last = 0;
      const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(60);
      while (std::chrono::steady_clock::now() < deadline) {
        const long r = vmm_chunks_ready(base);
        if (r < last || vmm_error(base)) {
          fail = true;
          return;
        }
        last = r;
        if (r >= target) return;
        std::this_thread::yield();
      }
      fail = true;  // no progress
    });
  for (auto& t : ts) t.join();
  CHECK(!fail.load());
}

int main() {
  int dev = 0;
  CHECK(hipSetDevice(dev) == hipSuccess);
  if (!vmm_supported(dev)) {
    std::printf("vmm not supported on this device: nothing to screen\n");
    return 0;
  }
  const long g = vmm_granularity(dev);
  CHECK(g > 0);
  const int regions = 4;
  const long chunks = 24, chunk = 2 * g, stride = chunks * chunk;

  // 1. async fill of every chunk while 4 threads poll; then zero-fill check on the GPU
  {
    void* base = nullptr;
    long reserved = 0;
    auto owner = vmm_reserve(stride * regions, dev, &base, &reserved);
    CHECK(owner && base && reserved >= stride * regions);
    CHECK(vmm_map_chunks(base, stride, regions, chunk, 0, 2, false));  // first chunks synchronously
    CHECK(vmm_chunks_ready(base) == 2);
    CHECK(vmm_map_chunks(base, stride, regions, chunk, 2, chunks - 2, true));
    CHECK(!vmm_map_chunks(base, stride, regions, chunk, 2, chunks - 2, true));  // one fill per arena
    poll_until(base, chunks, 4);
    unsigned* cnt = nullptr;
    CHECK(hipMalloc(&cnt, sizeof(unsigned)) == hipSuccess);
    CHECK(hipMemset(cnt, 0, sizeof(unsigned)) == hipSuccess);
    for (int r = 0; r < regions; ++r)
      count_nonzero<<<256, 256>>>(reinterpret_cast<const unsigned*>((char*)base + (size_t)r * stride),
                                  (size_t)stride / 4, cnt);
    unsigned h = 1;
    CHECK(hipMemcpy(&h, cnt, sizeof(unsigned), hipMemcpyDeviceToHost) == hipSuccess);
    CHECK(h == 0);
    CHECK(hipFree(cnt) == hipSuccess);
    vmm_forget(base);
    CHECK(vmm_chunks_ready(base) == -1);
  }  // owner dropped: unmap + release + address free

  // 2. drop the arena while its worker is mid-fill and other threads are looking it up:
  //    the destructor must stop + join the worker before anything is freed
  for (int rep = 0; rep < 4; ++rep) {
    void* base = nullptr;
    long reserved = 0;
    auto owner = vmm_reserve(stride * regions, dev, &base, &reserved);
    CHECK(owner);
    CHECK(vmm_map_chunks(base, stride, regions, chunk, 0, chunks, true));
    std::atomic<bool> go{true};
    std::vector<std::thread> lookers;
    for (int t = 0; t < 3; ++t)
      lookers.emplace_back([&] {
        while (go.load()) {
          (void)vmm_chunks_ready(base);  // -1 once forgotten: never a dangling arena
          (void)vmm_error(base);
        }
      });
    std::this_thread::sleep_for(std::chrono::microseconds(200 * rep));
    vmm_forget(base);
    owner.reset();
    go = false;
    for (auto& t : lookers) t.join();
  }

  // 3. several arenas filled concurrently (the global map under contention)
  {
    std::vector<std::shared_ptr<void>> owners(3);
    std::vector<void*> bases(3);
    for (int i = 0; i < 3; ++i) {
      long reserved = 0;
      owners[i] = vmm_reserve(stride * 2, dev, &bases[i], &reserved);
      CHECK(owners[i]);
      CHECK(vmm_map_chunks(bases[i], stride, 2, chunk, 0, chunks, true));
    }
    std::vector<std::thread> ts;
    for (int i = 0; i < 3; ++i) ts.emplace_back([&, i] { poll_until(bases[i], chunks, 2); });
    for (auto& t : ts) t.join();
    for (int i = 0; i < 3; ++i) vmm_forget(bases[i]);
  }
  CHECK(hipDeviceSynchronize() == hipSuccess);
  std::printf("vmm_stress ok (granularity %ld B, %d regions x %ld chunks)\n", g, regions, chunks);
  return 0;
}
