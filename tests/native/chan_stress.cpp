// Host-sanitizer screen of the TP step-header channel (ops/csrc/shm_channel.cc): one producer
// thread and N consumer threads on ONE mapping of the segment (so ThreadSanitizer sees every
// shared access at one address), far more messages than ring slots (the producer's back-pressure
// wait and the consumers' acquire loads both exercised), every consumer checks every message.
// Built by tests/test_native_sanitizers_cpu.py with -fsanitize=thread and with
// -fsanitize=address,undefined; exit 0 and no sanitizer report = pass.
#include <unistd.h>

#include <cstdio>
#include <string>
#include <thread>
#include <vector>

#include "shm_channel.cc"

int main(int argc, char** argv) {
  const int consumers = argc > 1 ? std::atoi(argv[1]) : 3;
  const long n = argc > 2 ? std::atol(argv[2]) : 20000;
  const std::string name = "/mlop-chan-stress-" + std::to_string(getpid());
  const long h = mlop::chan_create(name, 8, consumers);
  mlop::chan_unlink(name);
  std::vector<long> bad(consumers, 0);
  std::vector<std::thread> ts;
  for (int c = 0; c < consumers; ++c)
    ts.emplace_back([&, c] {
      int64_t w[9];
      for (long i = 0; i < n; ++i) {
        while (!mlop::chan_recv(h, c, w, 9, 1000)) {
        }
        for (int j = 0; j < 9; ++j) bad[c] += w[j] != 9 * i + j;
      }
    });
  int64_t w[9];
  for (long i = 0; i < n; ++i) {
    for (int j = 0; j < 9; ++j) w[j] = 9 * i + j;
    while (!mlop::chan_send(h, w, 9, 1000)) {
    }
  }
  for (auto& t : ts) t.join();
  mlop::chan_close(h, false);
  long total = 0;
  for (long b : bad) total += b;
  std::printf("consumers=%d messages=%ld mismatches=%ld\n", consumers, n, total);
  return total == 0 ? 0 : 1;
}
