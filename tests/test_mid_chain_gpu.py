"""Mid-M norm chain (5-64 rows, the canary's concurrency regime) on the planner's small tiles
(gemm.hip mid_chain_ok / launch_mid_res_ss / launch_mid_rs, rope_cache.hip's row-scaled slab
reduce): O / down split K and the tile's last split adds into the residual and leaves the row
sums of squares, gate_up / QKV scale their rows by the RMSNorm factor, so a decoder layer has no
add + RMSNorm launch.  Checked against the fp32 oracle and, for the residual, bit for bit against
the unfused split-K path (splitk_add_rmsnorm); relaunches are bit-identical; a 2-layer
Llama-3-8B-wide engine decodes the dense oracle's tokens with the chain on and off."""
import pytest
import torch

from mlopamd import ops
from mlopamd.ops import reference as ref

pytestmark = pytest.mark.gpu
bf = torch.bfloat16
H, I, EPS = 4096, 14336, 1e-5
MS = [5, 8, 9, 16, 17, 24, 33, 48, 64]


def close(a, b, atol=2e-2, rtol=2e-2):
    torch.testing.assert_close(a.float().cpu(), b.float().cpu(), atol=atol, rtol=rtol)


def _unit_norm(r):
    rf = r.float()
    return rf * torch.rsqrt(rf.pow(2).mean(-1, keepdim=True) + EPS)


@pytest.fixture(params=[1, 2], ids=["sc1", "acquire"])
def mid(gpu, request):
    """The mid chain on (it is off in serving, gemm_mid_chain 0: it measured slower end to end,
    profiles/r06_mid_chain.md), the weight-streaming decode chain off (5-64 rows are the mid
    chain's), the hand-written GEMM backend and the stream-K scratch the chain's tickets live in;
    the finishing split reads the partials with sc1 loads (1) or plain loads behind an acquire (2)."""
    ops.GEMM_BACKEND = "mlop"
    ops._sk_reserve(torch.device(gpu))
    prev_ws, prev_mid = torch.ops.mlop.gemm_ws_max_m(-1), torch.ops.mlop.gemm_mid_chain(-1)
    torch.ops.mlop.gemm_ws_max_m(0)
    torch.ops.mlop.gemm_mid_chain(request.param)
    try:
        yield
    finally:
        torch.ops.mlop.gemm_ws_max_m(prev_ws)
        torch.ops.mlop.gemm_mid_chain(prev_mid)
        ops.GEMM_BACKEND = ops.GEMM_BACKEND_DEFAULT


@pytest.mark.parametrize("K", [H, I], ids=["o", "down"])
@pytest.mark.parametrize("M", MS)
def test_mid_res_ss(gpu, mid, M, K):
    assert torch.ops.mlop.mid_chain_ok(M, H, K, 0)
    torch.manual_seed(M + K)
    a = torch.randn(M, K, device=gpu, dtype=bf)
    w = (0.02 * torch.randn(H, K, device=gpu)).to(bf)
    res = torch.randn(M, H, device=gpu, dtype=bf)
    r1, ss = res.clone(), ops.ss_buffer(M, H, gpu).fill_(float("nan"))
    ops.gemm_res_ss(a, w, r1, ss)
    exp = res.float() + a.float() @ w.float().t()
    close(r1, exp, atol=3e-2 * exp.abs().max().item() / 10 + 1e-2, rtol=2e-2)
    tot = ops.ss_parts(ss, M, H)[1]
    close(tot, r1.float().pow(2).sum(-1), atol=1e-2, rtol=1e-4)
    # the unfused path (split-K + splitk_add_rmsnorm) on the same plan: the residual bit for bit
    # (at 5-8 rows the O shape goes to the weight-streaming kernel there instead: another order)
    r2 = res.clone()
    ops.gemm_add_rmsnorm(a, w, r2, torch.ones(H, device=gpu, dtype=bf), EPS)
    if K == I or M > 8:
        assert torch.equal(r1, r2)
    else:
        close(r1, r2)
    # a relaunch re-arms every ticket and sums in the same fixed orders
    r3, ss3 = res.clone(), torch.empty_like(ss)
    ops.gemm_res_ss(a, w, r3, ss3)
    assert torch.equal(r1, r3) and torch.equal(tot, ops.ss_parts(ss3, M, H)[1])


@pytest.mark.parametrize("M", MS)
def test_mid_rs_silu(gpu, mid, M):
    assert torch.ops.mlop.mid_chain_ok(M, 2 * I, H, 1)
    torch.manual_seed(M)
    x = (3 * torch.randn(M, H, device=gpu)).to(bf)
    w = (0.02 * torch.randn(2 * I, H, device=gpu)).to(bf)
    ss = ops.ss_buffer(M, H, gpu).fill_(float("nan"))
    ops.ss_parts(ss, M, H)[1].copy_(x.float().pow(2).sum(-1))
    y = ops.gemm_rs(x, w, ss, EPS, ops.EPI_SILU_MUL)
    exp = ref.silu_mul(ops.deinterleave_cols((_unit_norm(x) @ w.float().t()).to(bf)))
    close(y, exp, atol=3e-2 * exp.abs().max().item() / 10 + 1e-2, rtol=3e-2)


@pytest.mark.parametrize("M", MS)
def test_mid_rs_rope(gpu, mid, M):
    """QKV + RoPE + paged K / V of the row-scaled residual: the weight-streaming kernel's RS
    prologue at 5-8 rows, the split-K slab reduce with the row factor above."""
    from mlopamd.models.layers import rope_table

    Hq, Hkv, D, BS = 32, 8, 128, 16
    N = (Hq + 2 * Hkv) * D
    assert torch.ops.mlop.mid_chain_ok(M, N, H, 3)
    NB = M // BS + 8
    torch.manual_seed(M)
    cs = rope_table(D, 8192, 5e5, device=gpu)
    x = (3 * torch.randn(M, H, device=gpu)).to(bf)
    w = (0.02 * torch.randn(N, H, device=gpu)).to(bf)
    pos = torch.randint(0, 8000, (M,), device=gpu, dtype=torch.int32)
    slots = torch.randperm(NB * BS, device=gpu)[:M].to(torch.int32)
    slots[M // 2] = -1
    ss = ops.ss_buffer(M, H, gpu).fill_(float("nan"))
    ops.ss_parts(ss, M, H)[1].copy_(x.float().pow(2).sum(-1))
    kc = torch.zeros(NB, Hkv, BS, D, device=gpu, dtype=bf)
    vc = torch.zeros(NB, Hkv, BS, D, device=gpu, dtype=bf)
    q = ops.qkv_rope_cache_rs(x, w, pos, cs, slots, kc, vc, Hq, ss, EPS)
    qkv_ref = (_unit_norm(x) @ w.float().t()).to(bf).cpu()
    kr, vr = torch.zeros_like(kc).cpu(), torch.zeros_like(vc).cpu()
    q_ref = ref.rope_cache(qkv_ref, pos.cpu(), cs.cpu(), slots.cpu(), kr, vr, Hq)
    close(q, q_ref)
    close(kc, kr)
    close(vc, vr)


@pytest.mark.parametrize("batch", [6, 16, 24, 64])
def test_llama_decode_mid_chain_on_off(gpu, mid, batch):
    """2-layer Llama-3-8B-wide engine, decode graphs on: batch 6 / 16 / 24 / 64 (6 and 24 replay
    the 8- / 32-row graphs with padding rows) with the mid chain (no add + RMSNorm launch in a
    layer) and without it both follow the fp32 dense oracle."""
    from mlopamd.models import build_model
    from mlopamd.models.config import get_config
    from mlopamd.models.reference import dense_logits
    from mlopamd.runtime.engine import Engine, EngineConfig
    from mlopamd.runtime.sampler import SamplingParams

    cfg = get_config("llama3-8b", num_layers=2)
    model = build_model(cfg, device=gpu, seed=7)
    prompts = [torch.randint(1000, 100000, (48,)).tolist() for _ in range(batch)]
    outs = {}
    mode = torch.ops.mlop.gemm_mid_chain(-1)
    for on in (0, 1):
        torch.ops.mlop.gemm_mid_chain(mode if on else 0)
        assert model._chain_ok(batch) == bool(on)
        ops._GEMM_USED.clear()  # before the engine: its graph captures run the decode forwards
        eng = Engine(model, EngineConfig(max_num_seqs=batch, max_num_batched_tokens=512, max_model_len=128,
                                         num_kv_blocks=batch * 8 + 1, use_graphs=True))
        outs[on] = eng.generate(prompts, SamplingParams(max_tokens=6, ignore_eos=True))
        assert eng.stats["graph_steps"] > 0
        small = set(k[3] for k in ops._GEMM_USED if 4 < k[0] <= 64)
        assert (ops.EPI_ADD_SS in small) == bool(on), small
    for on in (0, 1):
        for p, o in zip(prompts[:6], outs[on][:6]):
            toks = list(p)
            for t in o:
                lg = dense_logits(model, toks)[-1]
                best = int(lg.argmax())
                assert t == best or float(lg[best] - lg[t]) < 0.1 * float(lg.std()), (on, len(toks), best, t)
                toks.append(t)
