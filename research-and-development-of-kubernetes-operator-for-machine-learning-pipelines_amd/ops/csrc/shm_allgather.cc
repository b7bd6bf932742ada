// Host-to-host all-gather of a data-parallel-attention / expert-parallel group on one node
// (runtime/ep_serving.py EPGroupLoop, runtime/engine.py EPSync): every rank of the group
// contributes up to `max_words` int64 per exchange and receives every rank's contribution, over
// POSIX shared memory, in lock-step exchanges (every rank calls exchange() the same number of
// times in the same order).  It replaces the gloo TCP collectives of the EP serving loop -- a
// header / payload broadcast, two output all_gathers and the per-step MAX agreement, each a
// TCP round trip per iteration -- with one shared-memory hop each (a broadcast is an all-gather
// in which only the source's words are read).
//
//   [XgHeader | published[world] | done[world] | slots: world x nslots x (len + max_words)]
//   exchange i on rank r:
//     1. wait until every rank finished exchange i - nslots + 1 (done[q] >= i - nslots + 1): the
//        slot (r, i % nslots) is no longer read by anyone;
//     2. write len + words into slot (r, i % nslots), published[r].store(i + 1, release);
//     3. for every rank q: wait published[q] >= i + 1 (acquire), copy its slot;
//     4. done[r].store(i + 1, release).
// A rank can therefore run at most nslots - 1 exchanges ahead of the slowest one.  Every wait
// spins, yields, then sleeps (an idle serving group costs no host core) and is bounded by the
// caller's time slice; the call resumes where it stopped, and the caller's deadline turns a
// dead peer into an error instead of a hung predictor.
// Host code only (ops/build.py compiles csrc/*.cc as C++).
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

constexpr uint32_t kXgMagic = 0x6d6c7867u;  // "mlxg"
constexpr int kXgMaxRanks = 64;

struct alignas(64) XgCounter {
  std::atomic<int64_t> v;
  char pad[64 - sizeof(std::atomic<int64_t>)];
};

struct alignas(64) XgHeader {
  uint32_t magic, world, nslots, ready;
  int64_t max_words;
  char pad[64 - 4 * sizeof(uint32_t) - sizeof(int64_t)];
  XgCounter published[kXgMaxRanks];  // exchanges whose words rank q has written
  XgCounter done[kXgMaxRanks];       // exchanges rank q has finished reading
};

struct Xg {
  XgHeader* h = nullptr;
  int64_t* slots = nullptr;  // world x nslots x (1 + max_words)
  size_t bytes = 0;
  std::string name;
  bool owner = false;
  int rank = 0;
  int64_t iter = 0;  // exchanges this rank completed
  int phase = 0;     // 0: exchange `iter` not yet published; 1: published, reading rank next_q on
  int next_q = 0;
};

size_t xg_bytes(int world, int nslots, long max_words) {
  return sizeof(XgHeader) + (size_t)world * nslots * (size_t)(1 + max_words) * sizeof(int64_t);
}

Xg* xg_get(long hd) {
  if (hd == 0) throw std::runtime_error("shm all-gather: null handle");
  return reinterpret_cast<Xg*>(hd);
}

template <class F>
bool xg_wait(F ready, long timeout_us) {  // spin, yield (2 ms), 20 us sleeps (50 ms), 500 us sleeps
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

int64_t* xg_slot(Xg* x, int q, int64_t i) {
  const XgHeader* h = x->h;
  return x->slots + ((size_t)q * h->nslots + (size_t)(i % h->nslots)) * (size_t)(1 + h->max_words);
}

Xg* xg_map(const std::string& name, int fd, size_t bytes, bool owner, int rank) {
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    if (owner) shm_unlink(name.c_str());
    throw std::runtime_error("shm all-gather: mmap failed");
  }
  auto* x = new Xg;
  x->h = static_cast<XgHeader*>(p);
  x->slots = reinterpret_cast<int64_t*>(static_cast<char*>(p) + sizeof(XgHeader));
  x->bytes = bytes;
  x->name = name;
  x->owner = owner;
  x->rank = rank;
  return x;
}

}  // namespace

long xg_create(const std::string& name, int world, int nslots, long max_words) {
  if (world < 1 || world > kXgMaxRanks || nslots < 2 || max_words < 1)
    throw std::runtime_error("shm all-gather: bad sizes");
  const int fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0) throw std::runtime_error("shm all-gather: shm_open(create) failed for " + name);
  const size_t bytes = xg_bytes(world, nslots, max_words);
  if (ftruncate(fd, (off_t)bytes) != 0) {
    close(fd);
    shm_unlink(name.c_str());
    throw std::runtime_error("shm all-gather: ftruncate failed");
  }
  Xg* x = xg_map(name, fd, bytes, true, 0);
  std::memset(static_cast<void*>(x->h), 0, sizeof(XgHeader));  // the slots are zero from ftruncate
  x->h->world = (uint32_t)world;
  x->h->nslots = (uint32_t)nslots;
  x->h->max_words = max_words;
  x->h->magic = kXgMagic;
  std::atomic_thread_fence(std::memory_order_release);
  __atomic_store_n(&x->h->ready, 1u, __ATOMIC_RELEASE);
  return reinterpret_cast<long>(x);
}

long xg_open(const std::string& name, int rank) {
  const int fd = shm_open(name.c_str(), O_RDWR, 0600);
  if (fd < 0) throw std::runtime_error("shm all-gather: shm_open(open) failed for " + name);
  struct stat st {};
  if (fstat(fd, &st) != 0 || (size_t)st.st_size < sizeof(XgHeader)) {
    close(fd);
    throw std::runtime_error("shm all-gather: segment too small");
  }
  Xg* x = xg_map(name, fd, (size_t)st.st_size, false, rank);
  const XgHeader* h = x->h;
  if (__atomic_load_n(&h->ready, __ATOMIC_ACQUIRE) != 1u || h->magic != kXgMagic ||
      xg_bytes((int)h->world, (int)h->nslots, (long)h->max_words) != x->bytes || rank < 0 ||
      rank >= (int)h->world) {
    munmap(x->h, x->bytes);
    delete x;
    throw std::runtime_error("shm all-gather: not an initialised segment (or bad rank)");
  }
  return reinterpret_cast<long>(x);
}

long xg_max_words(long hd) { return (long)xg_get(hd)->h->max_words; }

// in: n words of this rank; out: world x max_words (row q = rank q's words); counts: world.
// Returns false when `timeout_us` expires first; the call is RESUMABLE: calling again continues
// the same exchange where it stopped (the words already published are not re-read from `in`),
// so the Python side waits in short slices and keeps its own overall deadline.
bool xg_exchange(long hd, const int64_t* in, long n, int64_t* out, int64_t* counts, long timeout_us) {
  Xg* x = xg_get(hd);
  XgHeader* h = x->h;
  const int W = (int)h->world, r = x->rank;
  const long mw = (long)h->max_words;
  const int64_t i = x->iter;
  if (x->phase == 0) {
    if (n < 0 || n > mw) throw std::runtime_error("shm all-gather: message larger than a slot");
    const int64_t need = i - (int64_t)h->nslots + 1;
    if (need > 0 && !xg_wait([&] {
          for (int q = 0; q < W; ++q)
            if (h->done[q].v.load(std::memory_order_acquire) < need) return false;
          return true;
        }, timeout_us))
      return false;
    int64_t* mine = xg_slot(x, r, i);
    mine[0] = n;
    if (n) std::memcpy(mine + 1, in, (size_t)n * sizeof(int64_t));
    h->published[r].v.store(i + 1, std::memory_order_release);
    x->phase = 1;
    x->next_q = 0;
  }
  for (int q = x->next_q; q < W; ++q) {
    if (!xg_wait([&] { return h->published[q].v.load(std::memory_order_acquire) >= i + 1; }, timeout_us)) {
      x->next_q = q;
      return false;
    }
    const int64_t* s = xg_slot(x, q, i);
    const int64_t len = s[0];
    if (len < 0 || len > mw) throw std::runtime_error("shm all-gather: corrupt slot length");
    counts[q] = len;
    if (len) std::memcpy(out + (size_t)q * mw, s + 1, (size_t)len * sizeof(int64_t));
  }
  h->done[r].v.store(i + 1, std::memory_order_release);
  x->iter = i + 1;
  x->phase = 0;
  return true;
}

void xg_close(long hd) {
  Xg* x = xg_get(hd);
  munmap(x->h, x->bytes);
  if (x->owner) shm_unlink(x->name.c_str());
  delete x;
}

}  // namespace mlop
