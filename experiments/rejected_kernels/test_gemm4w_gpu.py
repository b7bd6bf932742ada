"""K1 four-wave 256x256 GEMM body (ops/csrc/gemm4w.hip, planner variant 4) vs a plain fp32
PyTorch oracle: plain, SiLU-mul and QKV RoPE + paged-cache epilogues; ragged M, K from two
to 448 32-deep steps (ring wrap-around and the clamped tail re-loads), back-to-back launches."""
import pytest
import torch

from mlopamd import ops
from mlopamd.ops import reference as ref

pytestmark = pytest.mark.gpu
bf = torch.bfloat16


def close(a, b, atol, rtol):
    torch.testing.assert_close(a.float().cpu(), b.float().cpu(), atol=atol, rtol=rtol)


@pytest.fixture
def variant4(gpu):
    prev = torch.ops.mlop.gemm_big_variant(-1)
    torch.ops.mlop.gemm_big_variant(4)
    ops.GEMM_BACKEND = "mlop"
    yield gpu
    torch.ops.mlop.gemm_big_variant(prev)
    ops.GEMM_BACKEND = "auto"


@pytest.mark.parametrize("M,N,K", [(512, 256, 128), (600, 512, 192), (1000, 768, 4096), (2040, 6144, 4096),
                                   (4088, 4096, 4096), (1024, 4096, 14336), (777, 1280, 1024)])
def test_gemm4w_plain(variant4, M, N, K):
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device=variant4, dtype=bf)
    w = (0.05 * torch.randn(N, K, device=variant4)).to(bf)
    exp = x.float() @ w.float().t()
    tol = 3e-2 * exp.abs().max().item() / 10 + 1e-2
    for _ in range(2):  # back to back
        close(ops.gemm(x, w), exp, tol, 2e-2)


@pytest.mark.parametrize("M,I,K", [(512, 1024, 256), (2048, 14336, 4096), (1300, 640, 512)])
def test_gemm4w_silu_mul(variant4, M, I, K):
    torch.manual_seed(I)
    x = torch.randn(M, K, device=variant4, dtype=bf)
    g = (0.05 * torch.randn(I, K, device=variant4)).to(bf)
    u = (0.05 * torch.randn(I, K, device=variant4)).to(bf)
    y = ops.gemm(x, ops.interleave_gate_up(g, u), epi=ops.EPI_SILU_MUL)
    gu = (x.float() @ torch.cat([g, u]).float().t()).to(bf)
    close(y, ref.silu_mul(gu), 3e-2, 3e-2)


@pytest.mark.parametrize("M,Hq,Hkv", [(600, 32, 8), (2048, 32, 8), (4088, 32, 8), (1000, 8, 1)])
def test_gemm4w_qkv_rope(variant4, M, Hq, Hkv):
    from mlopamd.models.layers import rope_table

    D, K, BS = 128, 4096, 16
    N = (Hq + 2 * Hkv) * D
    if N % 256:
        pytest.skip("N not a multiple of 256")
    NB = M // BS + 8
    gpu = variant4
    cs = rope_table(D, 8192, 5e5, device=gpu)
    x = torch.randn(M, K, device=gpu, dtype=bf)
    w = (0.02 * torch.randn(N, K, device=gpu)).to(bf)
    pos = torch.randint(0, 8000, (M,), device=gpu, dtype=torch.int32)
    slots = torch.randperm(NB * BS, device=gpu)[:M].to(torch.int32)
    slots[5] = -1
    kc = torch.zeros(NB, Hkv, BS, D, device=gpu, dtype=bf)
    vc = torch.zeros(NB, Hkv, D, BS, device=gpu, dtype=bf)
    q = torch.empty(M, Hq, D, device=gpu, dtype=bf)
    assert torch.ops.mlop.gemm_rope_cache(q, kc, vc, x, w, pos, cs, slots)
    qkv_ref = (x.float() @ w.float().t()).to(bf).cpu()
    kr, vr = torch.zeros_like(kc).cpu(), torch.zeros_like(vc).cpu()
    q_ref = ref.rope_cache(qkv_ref, pos.cpu(), cs.cpu(), slots.cpu(), kr, vr, Hq)
    close(q, q_ref, 2e-2, 2e-2)
    close(kc, kr, 2e-2, 2e-2)
    close(vc, vr, 2e-2, 2e-2)
