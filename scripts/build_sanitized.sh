#!/bin/bash
# Host-side sanitizer builds of the native harnesses under tests/native/ (CPU container:
# hipcc cross-compiles for gfx950; the binaries run on the GPU box, see
# tests/test_native_sanitizers_gpu.py).  Sanitizers instrument HOST code only: every
# -fsanitize= sits directly after -Xarch_host (no GPU ASan / XNACK on this pool).
set -euo pipefail
cd "$(dirname "$0")/.."
out=build/native
mkdir -p "$out"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
common=(--offload-arch=gfx950 -std=c++17 -O1 -g -fno-omit-frame-pointer -pthread)
$HIPCC "${common[@]}" -Xarch_host -fsanitize=thread tests/native/vmm_stress.hip -o "$out/vmm_stress_tsan"
$HIPCC "${common[@]}" -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
  -Xarch_host -fno-sanitize-recover=undefined tests/native/vmm_stress.hip -o "$out/vmm_stress_asan"
$HIPCC "${common[@]}" tests/native/vmm_stress.hip -o "$out/vmm_stress_plain"
ls -la "$out"
# negative controls (host-only C++): the sanitizers must catch these
CXX=${CXX_SAN:-/opt/rocm/lib/llvm/bin/clang++}
$CXX -std=c++17 -O1 -g -pthread -fsanitize=thread tests/native/sanitizer_canary.cpp -o "$out/canary_tsan"
$CXX -std=c++17 -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=undefined \
  tests/native/sanitizer_canary.cpp -o "$out/canary_asan"
