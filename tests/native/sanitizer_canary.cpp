// Negative controls for the host-sanitizer screens: each mode has a deliberate defect the
// sanitizer must report (proves the runtime is linked and active with the flags used by
// scripts/build_sanitized.sh).  Built and run on CPU by tests/test_native_sanitizers_cpu.py.
#include <cstdio>
#include <cstring>
#include <thread>

static int shared_counter = 0;  // unsynchronised on purpose

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "race";
  if (!std::strcmp(mode, "race")) {
    std::thread a([] { for (int i = 0; i < 100000; ++i) ++shared_counter; });
    std::thread b([] { for (int i = 0; i < 100000; ++i) ++shared_counter; });
    a.join();
    b.join();
    std::printf("%d\n", shared_counter);
  } else if (!std::strcmp(mode, "uaf")) {
    int* p = new int[8];
    delete[] p;
    std::printf("%d\n", p[3]);  // heap-use-after-free
  } else if (!std::strcmp(mode, "ub")) {
    volatile int big = 0x7fffffff;
    std::printf("%d\n", big + argc);  // signed overflow
  }
  return 0;
}
