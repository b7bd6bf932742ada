"""GEMM backend autotune bookkeeping (host side, no GPU): row-count keys and the frozen
mode's nearest-tuned-key fallback used by serving loops and the benchmark's timed steps."""
from mlopamd import ops


def test_mbucket_keys():
    assert [ops._mbucket(m) for m in (1, 3, 64, 200, 256)] == [1, 4, 64, 256, 256]
    # above one 256-row tile: every 256 rows (the tile count decides the winner there)
    assert [ops._mbucket(m) for m in (257, 512, 2040, 2048, 2049, 4088)] == [512, 512, 2048, 2048, 2304, 4096]


def test_frozen_autotune_takes_nearest_tuned_rows(monkeypatch):
    monkeypatch.setattr(ops, "_GEMM_CHOICE", {(2048, 6144, 4096, 3): "hipblaslt", (4096, 6144, 4096, 3): "mlop",
                                              (2048, 4096, 4096, 0): "mlop"})
    assert ops._nearest_choice((2304, 6144, 4096, 3)) == "hipblaslt"
    assert ops._nearest_choice((3840, 6144, 4096, 3)) == "mlop"
    assert ops._nearest_choice((2304, 28672, 4096, 1)) is None  # no tuned key of that shape
    ops.freeze_autotune()
    try:
        assert ops.AUTOTUNE_FROZEN
    finally:
        ops.freeze_autotune(False)
    assert not ops.AUTOTUNE_FROZEN
