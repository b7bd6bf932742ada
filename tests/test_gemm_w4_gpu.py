"""Four-wave hand-scheduled GEMM (gemm_w4.hip: 256x256, planner variant 5, and the 128x256
half-height tile, variant 6) vs the fp32
PyTorch oracle: plain, SiLU-mul and RoPE + paged-cache epilogues, ragged M, persistent
workgroups walking 1-7 tiles (the next tile's first K-tiles prefetched under the epilogue
stores), the shortest K the peeled loop supports (192: first + nodma + last, no steady)."""
import pytest
import torch

from mlopamd import ops
from mlopamd.ops import reference as ref

pytestmark = pytest.mark.gpu
bf = torch.bfloat16


def close(a, b, atol=2e-2, rtol=2e-2):
    torch.testing.assert_close(a.float().cpu(), b.float().cpu(), atol=atol, rtol=rtol)


@pytest.fixture(params=[256, 128], ids=["bm256", "bm128"])
def w4(gpu, request):
    """The four-wave kernel at both tile heights: 256 x 256 (planner variant 5) and the
    128 x 256 half-height tile (variant 6, forced through the dense-plan override)."""
    prev = torch.ops.mlop.gemm_big_variant(-1)
    torch.ops.mlop.gemm_big_variant(5)
    if request.param == 128:
        torch.ops.mlop.gemm_dense_plan(6, 128, 256, -1)
    ops.GEMM_BACKEND = "mlop"
    try:
        yield request.param
    finally:
        torch.ops.mlop.gemm_dense_plan(-1, -1, -1, -1)
        torch.ops.mlop.gemm_big_variant(prev)
        ops.GEMM_BACKEND = ops.GEMM_BACKEND_DEFAULT


# every shape has >= 192 256x256 tiles (the planner's threshold for the 256x256 kernels)
@pytest.mark.parametrize("M,N,K", [(4096, 4096, 4096), (2048, 6144, 4096), (4088, 4096, 14336),
                                   (3000, 4096, 256), (3000, 4352, 192), (2100, 8448, 2048),
                                   (5000, 3072, 512), (4096, 16384, 1024), (4088, 28672, 320),
                                   # K-half tail items: 384 = 256 + 2 x 128, 128 -> 256 halves
                                   (4088, 6144, 4096), (2048, 4096, 4096), (2048, 4096, 14336)])
def test_w4_gemm(gpu, w4, M, N, K):
    torch.manual_seed(M + N + K)
    ops._sk_reserve(torch.device(gpu))  # the tail split's partial slots / tickets
    x = torch.randn(M, K, device=gpu, dtype=bf)
    w = (0.05 * torch.randn(N, K, device=gpu)).to(bf)
    y = ops.gemm(x, w)
    exp = x.float() @ w.float().t()
    close(y, exp, atol=3e-2 * exp.abs().max().item() / 10 + 1e-2, rtol=2e-2)
    y2 = ops.gemm(x, w)
    close(y, y2, atol=0, rtol=0)  # deterministic, no stale LDS between launches


@pytest.mark.parametrize("M,I,K", [(4088, 14336, 4096), (3000, 4096, 1024), (2040, 14336, 4096)])
def test_w4_silu_mul(gpu, w4, M, I, K):
    torch.manual_seed(M + I)
    ops._sk_reserve(torch.device(gpu))
    x = torch.randn(M, K, device=gpu, dtype=bf)
    w = (0.05 * torch.randn(2 * I, K, device=gpu)).to(bf)
    y = ops.gemm(x, w, epi=ops.EPI_SILU_MUL)
    exp = ref.silu_mul(ops.deinterleave_cols((x.float() @ w.float().t()).to(bf)))
    close(y, exp, atol=3e-2 * exp.abs().max().item() / 10 + 1e-2, rtol=3e-2)


@pytest.mark.parametrize("M,Hq,Hkv", [(2048, 32, 8), (3000, 32, 8), (4088, 32, 8), (4096, 16, 4)])
def test_w4_qkv_rope_cache(gpu, w4, M, Hq, Hkv):
    from mlopamd.models.layers import rope_table

    D, K, BS = 128, 4096, 16
    N = (Hq + 2 * Hkv) * D
    NB = M // BS + 8
    torch.manual_seed(M)
    ops._sk_reserve(torch.device(gpu))
    cs = rope_table(D, 8192, 5e5, device=gpu)
    x = torch.randn(M, K, device=gpu, dtype=bf)
    w = (0.02 * torch.randn(N, K, device=gpu)).to(bf)
    pos = torch.randint(0, 8000, (M,), device=gpu, dtype=torch.int32)
    slots = torch.randperm(NB * BS, device=gpu)[:M].to(torch.int32)
    slots[5] = -1
    slots[M - 1] = -1
    kc = torch.zeros(NB, Hkv, BS, D, device=gpu, dtype=bf)
    vc = torch.zeros(NB, Hkv, BS, D, device=gpu, dtype=bf)
    q = torch.empty(M, Hq, D, device=gpu, dtype=bf)
    assert torch.ops.mlop.gemm_rope_cache(q, kc, vc, x, w, pos, cs, slots)
    qkv_ref = (x.float() @ w.float().t()).to(bf).cpu()
    kr, vr = torch.zeros_like(kc).cpu(), torch.zeros_like(vc).cpu()
    q_ref = ref.rope_cache(qkv_ref, pos.cpu(), cs.cpu(), slots.cpu(), kr, vr, Hq)
    close(q, q_ref)
    close(kc, kr)
    close(vc, vr)
