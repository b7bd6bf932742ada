import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mlopamd import ops

    ops.load()  # must load: GPU tests never run on a silent fallback
    return torch.device("cuda", 0)


@pytest.fixture
def pp_variant(gpu):
    """Pin the large-M GEMM planner to the ping-pong kernel (variant 3: the one with the
    stream-K tail) for the test, whatever the default variant is."""
    import torch

    prev = torch.ops.mlop.gemm_big_variant(-1)
    torch.ops.mlop.gemm_big_variant(3)
    try:
        yield
    finally:
        torch.ops.mlop.gemm_big_variant(prev)


@pytest.fixture
def attn_fused_all(gpu):
    """Lift the (tile, kv head) pair cap of paged attention's in-launch split-KV combine (none
    by default; the op sets it) so a test's part_sem launch takes the fused path at any size."""
    import torch

    prev = torch.ops.mlop.attn_fused_max_pairs(1 << 30)
    try:
        yield
    finally:
        torch.ops.mlop.attn_fused_max_pairs(prev)
