"""Host-side sanitizer screens of the runtime's multi-threaded native code (GPU box).

``tests/native/vmm_stress.hip`` drives the lazily backed KV arena (ops/csrc/vmm.hip:
worker thread backing chunks, pollers, the global arena map, drop-while-filling) from
several threads; ``scripts/build_sanitized.sh`` (run by ``__graft_entry__.build()``)
builds it with ThreadSanitizer, with AddressSanitizer + UBSan (host code only: each
``-fsanitize=`` follows ``-Xarch_host``) and plain.  Each binary must exit 0 with no
sanitizer report.  Suppressions (tests/native/*.supp) cover only the uninstrumented ROCm
runtime libraries.  SURVEY.md §5 "race detection / sanitizers"."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "native")
SUPP = os.path.join(ROOT, "tests", "native")


@pytest.mark.parametrize("variant", ["plain", "tsan", "asan"])
def test_vmm_arena_under_sanitizers(variant):
    exe = os.path.join(BIN, f"vmm_stress_{variant}")
    if not os.path.exists(exe):
        pytest.fail(f"{exe} missing: run scripts/build_sanitized.sh (part of __graft_entry__.build())")
    env = dict(os.environ)
    env["TSAN_OPTIONS"] = f"halt_on_error=1 exitcode=66 second_deadlock_stack=1 suppressions={SUPP}/tsan.supp"
    env["ASAN_OPTIONS"] = "halt_on_error=1:exitcode=67:detect_leaks=1:protect_shadow_gap=0"
    env["LSAN_OPTIONS"] = f"suppressions={SUPP}/lsan.supp"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    r = subprocess.run([exe], env=env, capture_output=True, text=True, timeout=150)
    log = r.stdout + r.stderr
    assert r.returncode == 0 and "vmm_stress ok" in r.stdout, log[-4000:]
    for marker in ("WARNING: ThreadSanitizer", "ERROR: AddressSanitizer", "ERROR: LeakSanitizer",
                   "runtime error:"):
        assert marker not in log, log[-4000:]
