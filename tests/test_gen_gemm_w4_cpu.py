"""The four-wave GEMM's asm K-loop is generated (ops/gen_gemm_w4.py -> csrc/gemm_w4_asm.h):
the committed header must be exactly what the generator renders, and the generated loop must
keep its own invariants (the LDS queue across the back-edge, balanced barriers, vmcnt counts,
no scalar-cache writes)."""
import re

from mlopamd.ops import gen_gemm_w4 as gen


def test_header_matches_generator():
    assert gen.OUT.read_text() == gen.render(), "run: python -m mlopamd.ops.gen_gemm_w4"


def test_loop_invariants():
    for sc in gen.SCHEDS:
        for ns in (32, 16, 34, 18):
            lines = gen.kloop(ns, sc)
            text = "\n".join(lines)
            # 128 MFMAs per K-tile body: first + steady + nodma + last = 4 bodies
            assert sum(1 for ln in lines if ln.startswith("v_mfma")) == 4 * 128
            # 32 fragment reads per body, 16 more in the prologue; the last body reads no next tile
            assert sum(1 for ln in lines if ln.startswith("ds_read_b128")) == 16 + 3 * 32 + 16
            # every wave executes the same barriers: none inside a data-dependent branch
            assert text.count("s_barrier") == 1 + 2 * 2 + 1 + 1  # entry, first / steady B1 + B2, nodma B2, exit
            # the entry wait with a prefetched tile covers exactly the epilogue's stores
            assert f"s_waitcnt vmcnt({16 + ns})" in text
            # never a scalar-cache write of any form
            assert not re.search(r"\bs_(store|atomic|dcache_wb|dcache_discard|buffer_store)", text)
            # zero-C MFMAs only in the first body (64 of them)
            assert sum(1 for ln in lines if ln.startswith("v_mfma") and ln.endswith(", 0")) == 64
