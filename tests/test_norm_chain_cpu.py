"""Norm chain plumbing on CPU (ops' torch reference, MLOP_NORM_CHAIN=force): the large-M TP=1
forward without add + RMSNorm passes (O / down add into the residual and leave row partials,
gate_up / QKV scale their rows after the GEMM) generates what the dense oracle does, and
fold_norms() keeps the function of a model with non-unit norm weights."""
import pytest
import torch

from mlopamd import ops
from mlopamd.models import build_model
from mlopamd.models.config import TINY_LLAMA
from mlopamd.models.reference import dense_logits
from mlopamd.runtime.engine import Engine, EngineConfig
from mlopamd.runtime.sampler import SamplingParams


@pytest.fixture
def force_chain(monkeypatch):
    monkeypatch.setattr(ops, "NORM_CHAIN", "force")


def _greedy(model, prompt, n):
    toks, out = list(prompt), []
    for _ in range(n):
        t = int(dense_logits(model, toks)[-1].argmax())
        out.append(t)
        toks.append(t)
    return out


def test_chain_ops_match_add_rmsnorm(force_chain):
    torch.manual_seed(0)
    M, H, N = 7, 256, 384
    a, w = torch.randn(M, H), torch.randn(H, H) * 0.05
    res = torch.randn(M, H)
    g_w = torch.randn(N, H) * 0.05
    # reference: residual += a @ w^T; x = rmsnorm(residual); y = x @ g_w^T
    r_ref = res + a @ w.t()
    x_ref = r_ref * torch.rsqrt(r_ref.pow(2).mean(-1, keepdim=True) + 1e-5)
    r = res.clone()
    ss = ops.ss_buffer(M, H, "cpu")
    ops.gemm_res_ss(a, w, r, ss)
    torch.testing.assert_close(r, r_ref, rtol=1e-5, atol=1e-5)
    part, tot = ops.ss_parts(ss, M, H)
    torch.testing.assert_close(part.sum(-1), r_ref.pow(2).sum(-1), rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(tot, r_ref.pow(2).sum(-1), rtol=1e-5, atol=1e-4)
    y = ops.gemm_rs(r, g_w, ss, 1e-5)
    torch.testing.assert_close(y, x_ref @ g_w.t(), rtol=1e-4, atol=1e-4)


def test_chain_forward_generates_dense_tokens(force_chain):
    torch.manual_seed(0)
    model = build_model(TINY_LLAMA, device="cpu", dtype=torch.float32, seed=1)
    assert model.unit_norms and model._chain_ok(16)
    eng = Engine(model, EngineConfig(max_num_seqs=8, max_num_batched_tokens=64, max_model_len=256,
                                     num_kv_blocks=64, use_graphs=False))
    prompts = [torch.randint(2, 500, (n,)).tolist() for n in (5, 33, 17)]
    outs = eng.generate(prompts, SamplingParams(max_tokens=5, ignore_eos=True))
    for p, o in zip(prompts, outs):
        assert o == _greedy(model, p, 5)


def test_fold_norms_keeps_the_function():
    torch.manual_seed(0)
    model = build_model(TINY_LLAMA, device="cpu", dtype=torch.float32, seed=1)
    for L in model.layers:
        L["in_norm"].uniform_(0.5, 1.5)
        L["post_norm"].uniform_(0.5, 1.5)
    model.unit_norms = False
    assert not model._chain_ok(16)
    toks = torch.randint(2, 500, (12,)).tolist()
    before = dense_logits(model, toks)
    model.fold_norms()
    assert model.unit_norms
    torch.testing.assert_close(dense_logits(model, toks), before, rtol=1e-4, atol=1e-4)


def test_ss_init_and_all_reduce_add_fallback():
    """The decode chain's CPU pieces: ss_init fills the torch reference's row partials / totals
    (the GPU GEMV form ignores them), and Group.all_reduce_add without the K15 buffers adds
    the (here single-rank) sum into the residual with the kernel's rounding,
    bf16(residual + bf16(sum))."""
    from mlopamd.parallel.comm import Group

    torch.manual_seed(0)
    M, H = 3, 256
    x = (3 * torch.randn(M, H)).to(torch.bfloat16)
    ss = ops.ss_init(x, ops.ss_buffer(M, H, "cpu").fill_(float("nan")))
    part, tot = ops.ss_parts(ss, M, H)
    torch.testing.assert_close(part, x.float().pow(2).view(M, H // 128, 128).sum(-1))
    torch.testing.assert_close(tot, x.float().pow(2).sum(-1))
    res = torch.randn(M, H).to(torch.bfloat16)
    y = torch.randn(M, H).to(torch.bfloat16)
    exp = (res.float() + y.float()).to(torch.bfloat16)
    out = Group().all_reduce_add(y.clone(), res)
    assert out is res and torch.equal(res, exp)
