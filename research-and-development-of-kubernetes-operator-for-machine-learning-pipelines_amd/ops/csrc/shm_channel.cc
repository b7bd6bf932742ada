// Host-to-host step-header channel of a tensor-parallel group on one node (runtime/engine.py
// StepSync): a POSIX shared-memory broadcast ring with ONE producer (the TP leader, which alone
// schedules) and N-1 consumers (the worker ranks).  Each engine step the leader publishes a
// 9-int header; a worker learns it about a microsecond later (vs ~50-100 us for a gloo TCP
// broadcast) and enqueues that step's forward while the device still runs the previous one.
//
//   [ChanHeader | nslots x 128-B slots]
//   producer: wait until the slowest consumer is < nslots behind, copy the words into slot
//             seq % nslots, then seq.store(seq + 1, release);
//   consumer: spin (pause, then yield, then sleep) until seq > its own count (acquire), copy the slot, then
//             its ack.store(count + 1, release) -- every counter on its own cache line.
// Both sides take a timeout (microseconds) and return false when it expires, so the Python
// loop around them never blocks inside a C++ call indefinitely (and drops the GIL in between).
// Host code only: built with the extension (ops/build.py compiles csrc/*.cc as C++).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

namespace mlop {

namespace {

constexpr uint32_t kMagic = 0x6d6c6f70u;  // "mlop"
constexpr int kWords = 16;                // int64 per slot (one 128-B slot)
constexpr int kMaxConsumers = 63;

struct alignas(64) Counter {
  std::atomic<int64_t> v;
  char pad[64 - sizeof(std::atomic<int64_t>)];
};

struct alignas(128) ChanHeader {  // a multiple of 128 B: the slots after it stay 128-B aligned
  uint32_t magic, nslots, nconsumers, ready;
  char pad0[64 - 4 * sizeof(uint32_t)];
  Counter seq;                   // messages published
  Counter acks[kMaxConsumers];   // per consumer: messages consumed
};

struct alignas(128) Slot {
  int64_t w[kWords];
};
static_assert(sizeof(ChanHeader) % alignof(Slot) == 0, "slot alignment");

struct Chan {
  ChanHeader* h = nullptr;
  Slot* slots = nullptr;
  size_t bytes = 0;
  std::string name;
  bool owner = false;
};

size_t chan_bytes(int nslots) { return sizeof(ChanHeader) + (size_t)nslots * sizeof(Slot); }

Chan* get(long hd) {
  if (hd == 0) throw std::runtime_error("shm channel: null handle");
  return reinterpret_cast<Chan*>(hd);
}

// spin briefly (a step header is expected within microseconds), then yield the core, then
// back off to short sleeps: a parked worker of an idle predictor must not hold a host core at
// 100 % (7 cores at TP = 8).  Up to 2 ms of waiting: yield (sub-microsecond wake-up); up to
// 50 ms: 20 us sleeps (the header of a step still arrives well ahead of its device work under
// one-step-ahead scheduling); beyond: 500 us sleeps (an idle group).
template <class F>
bool wait_until(F ready, long timeout_us) {
  const auto t0 = std::chrono::steady_clock::now();
  for (long i = 0;; ++i) {
    if (ready()) return true;
    if (i < 4096) {
      __builtin_ia32_pause();
      continue;
    }
    const long waited =
        (long)std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
    if (waited >= timeout_us) return false;
    if (waited < 2000)
      std::this_thread::yield();
    else
      std::this_thread::sleep_for(std::chrono::microseconds(waited < 50000 ? 20 : 500));
  }
}

}  // namespace

long chan_create(const std::string& name, int nslots, int nconsumers) {
  if (nslots < 2 || nconsumers < 0 || nconsumers > kMaxConsumers) throw std::runtime_error("shm channel: bad sizes");
  const int fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0) throw std::runtime_error("shm channel: shm_open(create) failed for " + name);
  const size_t bytes = chan_bytes(nslots);
  if (ftruncate(fd, (off_t)bytes) != 0) {
    close(fd);
    shm_unlink(name.c_str());
    throw std::runtime_error("shm channel: ftruncate failed");
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    shm_unlink(name.c_str());
    throw std::runtime_error("shm channel: mmap failed");
  }
  std::memset(p, 0, bytes);
  auto* c = new Chan;
  c->h = static_cast<ChanHeader*>(p);
  c->slots = reinterpret_cast<Slot*>(static_cast<char*>(p) + sizeof(ChanHeader));
  c->bytes = bytes;
  c->name = name;
  c->owner = true;
  c->h->nslots = (uint32_t)nslots;
  c->h->nconsumers = (uint32_t)nconsumers;
  c->h->magic = kMagic;
  std::atomic_thread_fence(std::memory_order_release);
  __atomic_store_n(&c->h->ready, 1u, __ATOMIC_RELEASE);
  return reinterpret_cast<long>(c);
}

long chan_open(const std::string& name) {
  const int fd = shm_open(name.c_str(), O_RDWR, 0600);
  if (fd < 0) throw std::runtime_error("shm channel: shm_open(open) failed for " + name);
  struct stat st {};
  if (fstat(fd, &st) != 0 || (size_t)st.st_size < sizeof(ChanHeader)) {
    close(fd);
    throw std::runtime_error("shm channel: segment too small");
  }
  void* p = mmap(nullptr, (size_t)st.st_size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) throw std::runtime_error("shm channel: mmap failed");
  auto* h = static_cast<ChanHeader*>(p);
  if (__atomic_load_n(&h->ready, __ATOMIC_ACQUIRE) != 1u || h->magic != kMagic ||
      chan_bytes((int)h->nslots) != (size_t)st.st_size) {
    munmap(p, (size_t)st.st_size);
    throw std::runtime_error("shm channel: not an initialised channel");
  }
  auto* c = new Chan;
  c->h = h;
  c->slots = reinterpret_cast<Slot*>(static_cast<char*>(p) + sizeof(ChanHeader));
  c->bytes = (size_t)st.st_size;
  c->name = name;
  return reinterpret_cast<long>(c);
}

bool chan_send(long hd, const int64_t* w, int n, long timeout_us) {
  Chan* c = get(hd);
  if (n < 0 || n > kWords) throw std::runtime_error("shm channel: message larger than a slot");
  ChanHeader* h = c->h;
  const int64_t s = h->seq.v.load(std::memory_order_relaxed);  // single producer
  const int64_t ns = h->nslots;
  auto room = [&] {
    for (uint32_t i = 0; i < h->nconsumers; ++i)
      if (s - h->acks[i].v.load(std::memory_order_acquire) >= ns) return false;
    return true;
  };
  if (!wait_until(room, timeout_us)) return false;
  Slot& sl = c->slots[s % ns];
  std::memcpy(sl.w, w, (size_t)n * sizeof(int64_t));
  h->seq.v.store(s + 1, std::memory_order_release);
  return true;
}

bool chan_recv(long hd, int consumer, int64_t* w, int n, long timeout_us) {
  Chan* c = get(hd);
  ChanHeader* h = c->h;
  if (consumer < 0 || consumer >= (int)h->nconsumers) throw std::runtime_error("shm channel: bad consumer index");
  if (n < 0 || n > kWords) throw std::runtime_error("shm channel: message larger than a slot");
  const int64_t mine = h->acks[consumer].v.load(std::memory_order_relaxed);  // only this consumer writes it
  if (!wait_until([&] { return h->seq.v.load(std::memory_order_acquire) > mine; }, timeout_us)) return false;
  std::memcpy(w, c->slots[mine % (int64_t)h->nslots].w, (size_t)n * sizeof(int64_t));
  h->acks[consumer].v.store(mine + 1, std::memory_order_release);
  return true;
}

void chan_unlink(const std::string& name) { shm_unlink(name.c_str()); }

void chan_close(long hd, bool unlink) {
  Chan* c = get(hd);
  munmap(c->h, c->bytes);
  if (unlink || c->owner) shm_unlink(c->name.c_str());
  delete c;
}

}  // namespace mlop
