"""Negative controls for the host-sanitizer screens (tests/test_native_sanitizers_gpu.py):
with the same flags as scripts/build_sanitized.sh, ThreadSanitizer must report a planted
data race, AddressSanitizer a heap use-after-free and UBSan a signed overflow.  A screen
that cannot fail proves nothing; these show the runtimes are linked and active."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "native")
CXX = "/opt/rocm/lib/llvm/bin/clang++"
SRC = os.path.join(ROOT, "tests", "native", "sanitizer_canary.cpp")


def _canary(kind):
    exe = os.path.join(BIN, f"canary_{kind}")
    if not os.path.exists(exe):
        if not os.path.exists(CXX):
            pytest.skip("ROCm clang++ not available")
        os.makedirs(BIN, exist_ok=True)
        flags = ["-fsanitize=thread"] if kind == "tsan" else ["-fsanitize=address,undefined",
                                                               "-fno-sanitize-recover=undefined"]
        subprocess.run([CXX, "-std=c++17", "-O1", "-g", "-pthread", *flags, SRC, "-o", exe], check=True)
    return exe


@pytest.mark.parametrize("kind,mode,marker", [
    ("tsan", "race", "WARNING: ThreadSanitizer: data race"),
    ("asan", "uaf", "ERROR: AddressSanitizer: heap-use-after-free"),
    ("asan", "ub", "runtime error: signed integer overflow"),
])
def test_sanitizer_catches_planted_defect(kind, mode, marker):
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66", ASAN_OPTIONS="detect_leaks=0")
    r = subprocess.run([_canary(kind), mode], env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode != 0, r.stdout + r.stderr
    assert marker in r.stderr, r.stderr[-2000:]


@pytest.mark.parametrize("kind", ["tsan", "asan"])
def test_host_channel_under_sanitizers(kind, tmp_path):
    """The native TP header channel (ops/csrc/shm_channel.cc) under ThreadSanitizer and
    ASan + UBSan: one producer, three consumer threads on one mapping, 20k messages through an
    8-slot ring -- clean exit, every message intact, no sanitizer report."""
    if not os.path.exists(CXX):
        pytest.skip("ROCm clang++ not available")
    src = os.path.join(ROOT, "tests", "native", "chan_stress.cpp")
    inc = os.path.join(ROOT, "research-and-development-of-kubernetes-operator-for-machine-learning-pipelines_amd",
                       "ops", "csrc")
    exe = str(tmp_path / f"chan_{kind}")
    flags = ["-fsanitize=thread"] if kind == "tsan" else ["-fsanitize=address,undefined",
                                                           "-fno-sanitize-recover=undefined"]
    subprocess.run([CXX, "-std=c++17", "-O1", "-g", "-pthread", f"-I{inc}", *flags, src, "-o", exe], check=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66", ASAN_OPTIONS="detect_leaks=0")
    r = subprocess.run([exe, "3", "20000"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "mismatches=0" in r.stdout and "Sanitizer" not in r.stderr, r.stderr[-3000:]
