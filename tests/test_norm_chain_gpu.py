"""Norm chain on the four-wave GEMM (gemm_w4.hip W4_ADD_SS / W4_RS) vs the fp32 PyTorch
oracle at the Llama-3-8B shapes: O / down add into the residual in place and write per-row,
per-128-column sums of squares; gate_up (SiLU-mul) and QKV (RoPE + paged cache) read the raw
residual and scale each accumulator row by rsqrt(sum / K + eps).  Also: bit-identical
relaunches (partials are written, never accumulated) and a 2-layer 8B forward with the chain
on vs off."""
import pytest
import torch

from mlopamd import ops
from mlopamd.ops import reference as ref

pytestmark = pytest.mark.gpu
bf = torch.bfloat16
H, I, EPS = 4096, 14336, 1e-5


@pytest.fixture
def ws_on():
    """The decode chain's weight-streaming MFMA form (5-64 rows) is off in serving
    (gemm_ws_max_m = 0): on for these tests."""
    prev = torch.ops.mlop.gemm_ws_max_m(-1)
    torch.ops.mlop.gemm_ws_max_m(64)
    yield
    torch.ops.mlop.gemm_ws_max_m(prev)


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
    ops._sk_reserve(torch.device(gpu))
    try:
        yield request.param
    finally:
        torch.ops.mlop.gemm_dense_plan(-1, -1, -1, -1)
        torch.ops.mlop.gemm_big_variant(prev)
        ops.GEMM_BACKEND = ops.GEMM_BACKEND_DEFAULT


def _unit_norm(r):
    rf = r.float()
    return rf * torch.rsqrt(rf.pow(2).mean(-1, keepdim=True) + EPS)


@pytest.mark.parametrize("M,K", [(4088, H), (2048, H), (4088, I), (2040, I)])
def test_gemm_res_ss(gpu, w4, M, K):
    torch.manual_seed(M + K)
    assert torch.ops.mlop.w4_chain_ok(M, H, K)
    a = torch.randn(M, K, device=gpu, dtype=bf)
    w = (0.02 * torch.randn(H, K, device=gpu)).to(bf)
    res = torch.randn(M, H, device=gpu, dtype=bf)
    exp = res.float() + a.float() @ w.float().t()
    r = res.clone()
    ss = ops.ss_buffer(M, H, gpu).fill_(float("nan"))
    ops.gemm_res_ss(a, w, r, ss)
    close(r, exp, atol=3e-2 * exp.abs().max().item() / 10 + 1e-2, rtol=2e-2)
    # the partials are the sums of squares of the STORED (bf16) residual, group by group, and
    # the totals their row sums (the band's last tile)
    part, tot = ops.ss_parts(ss, M, H)
    close(part, r.float().pow(2).view(M, H // 128, 128).sum(-1), atol=1e-3, rtol=1e-4)
    close(tot, r.float().pow(2).sum(-1), atol=1e-2, rtol=1e-4)
    r2, ss2 = res.clone(), torch.empty_like(ss)
    ops.gemm_res_ss(a, w, r2, ss2)
    assert torch.equal(r, r2) and torch.equal(ss, ss2)  # deterministic


@pytest.mark.parametrize("M", [4088, 2048])
def test_gemm_rs_silu(gpu, w4, M):
    torch.manual_seed(M)
    x = (3 * torch.randn(M, H, device=gpu)).to(bf)
    w = (0.02 * torch.randn(2 * I, H, device=gpu)).to(bf)
    ss = ops.ss_buffer(M, H, gpu).fill_(float("nan"))
    ops.ss_parts(ss, M, H)[1].copy_(x.float().pow(2).sum(-1))
    y = ops.gemm_rs(x, w, ss, EPS, ops.EPI_SILU_MUL)
    exp = ref.silu_mul(ops.deinterleave_cols((_unit_norm(x) @ w.float().t()).to(bf)))
    close(y, exp, atol=3e-2 * exp.abs().max().item() / 10 + 1e-2, rtol=3e-2)


@pytest.mark.parametrize("M", [4088, 2048])
def test_gemm_rs_rope(gpu, w4, M):
    from mlopamd.models.layers import rope_table

    Hq, Hkv, D, BS = 32, 8, 128, 16
    N = (Hq + 2 * Hkv) * D
    NB = M // BS + 8
    torch.manual_seed(M)
    cs = rope_table(D, 8192, 5e5, device=gpu)
    x = (3 * torch.randn(M, H, device=gpu)).to(bf)
    w = (0.02 * torch.randn(N, H, device=gpu)).to(bf)
    pos = torch.randint(0, 8000, (M,), device=gpu, dtype=torch.int32)
    slots = torch.randperm(NB * BS, device=gpu)[:M].to(torch.int32)
    slots[7] = -1
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


def test_llama_forward_chain_on_off(gpu, w4, monkeypatch):
    """2-layer Llama-3-8B-wide forward over a 2048-token prefill batch: the chain (no add +
    RMSNorm launches between the projections) and the unfused layers agree to bf16 noise."""
    from mlopamd.models import build_model
    from mlopamd.models.config import get_config
    from mlopamd.models.reference import dense_logits
    from mlopamd.runtime.engine import Engine, EngineConfig
    from mlopamd.runtime.sampler import SamplingParams

    cfg = get_config("llama3-8b", num_layers=2)
    model = build_model(cfg, device=gpu, seed=5)
    assert model._chain_ok(2048)
    prompts = [torch.randint(1000, 100000, (256,)).tolist() for _ in range(8)]
    outs = {}
    for mode in ("0", "1"):
        monkeypatch.setattr(ops, "NORM_CHAIN", mode)
        eng = Engine(model, EngineConfig(max_num_seqs=8, max_num_batched_tokens=2048, max_model_len=512,
                                         num_kv_blocks=8 * 32 + 1, use_graphs=False))
        ops._GEMM_USED.clear()
        outs[mode] = eng.generate(prompts, SamplingParams(max_tokens=2, ignore_eos=True))
        used = set(k[3] for k in ops._GEMM_USED)
        assert (ops.EPI_ADD_SS in used) == (mode == "1"), used
    # both against the fp32 dense oracle (first token: the 2048-row chain step; second: decode)
    for mode in ("0", "1"):
        for p, o in zip(prompts[:4], outs[mode][:4]):
            toks = list(p)
            for t in o:
                lg = dense_logits(model, toks)[-1]
                best = int(lg.argmax())
                assert t == best or float(lg[best] - lg[t]) < 0.1 * float(lg.std()), (mode, len(toks), best, t)
                toks.append(t)


@pytest.mark.parametrize("M", [1, 2, 3, 4, 5, 8, 16, 17, 33, 48, 64])
def test_gemv_chain_res_rs(gpu, w4, ws_on, M):
    """Decode form of the chain (M <= 4: gemv.hip EPI_RES / PRO_RS; 5-64 rows: the
    weight-streaming MFMA kernel, gemm_ws.hip WS_RES / RS): O / down add into the residual in
    place with norm.hip's rounding, gate_up / plain / QKV + RoPE scale each row by
    rsqrt(mean(a^2) + eps) of the residual they stream.  The ss buffers are NaN: the decode
    form must neither read nor need them (the four-wave form would turn them into NaNs)."""
    from mlopamd.models.layers import rope_table

    torch.manual_seed(M)
    for K in (H, I):  # O (K = q_size = H) and down (K = I)
        assert torch.ops.mlop.gemv_chain_supported(M, H, K, 0)
        a = torch.randn(M, K, device=gpu, dtype=bf)
        w = (0.02 * torch.randn(H, K, device=gpu)).to(bf)
        res = torch.randn(M, H, device=gpu, dtype=bf)
        exp = (res.float() + (a.float() @ w.float().t()).to(bf).float()).to(bf)
        r, ss = res.clone(), ops.ss_buffer(M, H, gpu).fill_(float("nan"))
        ops.gemm_res_ss(a, w, r, ss)
        close(r, exp, atol=2e-2, rtol=1e-2)
        r2 = res.clone()
        ops.gemm_res_ss(a, w, r2, ss)
        assert torch.equal(r, r2)
    x = (3 * torch.randn(M, H, device=gpu)).to(bf)
    ss = ops.ss_buffer(M, H, gpu).fill_(float("nan"))
    w = (0.02 * torch.randn(2 * I, H, device=gpu)).to(bf)
    y = ops.gemm_rs(x, w, ss, EPS, ops.EPI_SILU_MUL)
    exp = ref.silu_mul(ops.deinterleave_cols((_unit_norm(x) @ w.float().t()).to(bf)))
    close(y, exp, atol=3e-2 * exp.abs().max().item() / 10 + 1e-2, rtol=3e-2)
    w = (0.02 * torch.randn(1024, H, device=gpu)).to(bf)
    y = ops.gemm_rs(x, w, ss, EPS, ops.EPI_NONE)
    close(y, (_unit_norm(x) @ w.float().t()).to(bf), atol=2e-2, rtol=2e-2)
    Hq, Hkv, D, BS = 32, 8, 128, 16
    N, NB = (Hq + 2 * Hkv) * D, 64
    cs = rope_table(D, 8192, 5e5, device=gpu)
    w = (0.02 * torch.randn(N, H, device=gpu)).to(bf)
    pos = torch.randint(0, 8000, (M,), device=gpu, dtype=torch.int32)
    slots = torch.randperm(NB * BS, device=gpu)[:M].to(torch.int32)
    if M > 1:
        slots[1] = -1  # a padding row: q only, no cache stores
    kc = torch.zeros(NB, Hkv, BS, D, device=gpu, dtype=bf)
    vc = torch.zeros(NB, Hkv, BS, D, device=gpu, dtype=bf)
    q = ops.qkv_rope_cache_rs(x, w, pos, cs, slots, kc, vc, Hq, ss, EPS)
    qkv_ref = (_unit_norm(x) @ w.float().t()).to(bf).cpu()
    kr, vr = torch.zeros_like(kc).cpu(), torch.zeros_like(vc).cpu()
    q_ref = ref.rope_cache(qkv_ref, pos.cpu(), cs.cpu(), slots.cpu(), kr, vr, Hq)
    close(q, q_ref)
    close(kc, kr)
    close(vc, vr)


@pytest.mark.parametrize("batch", [1, 3, 4, 8, 24])
def test_llama_decode_gemv_chain_on_off(gpu, w4, ws_on, monkeypatch, batch):
    """2-layer Llama-3-8B-wide engine, graphs on: decode steps of 1 / 3 / 4 sequences with the
    GEMV chain, of 8 / 24 with the weight-streaming MFMA chain (five launches per layer, no add
    + RMSNorm; batch 3 / 24 replay the 4- / 32-row graphs with padding rows) and without the
    chain all follow the fp32 dense oracle."""
    from mlopamd.models import build_model
    from mlopamd.models.config import get_config
    from mlopamd.models.reference import dense_logits
    from mlopamd.runtime.engine import Engine, EngineConfig
    from mlopamd.runtime.sampler import SamplingParams

    cfg = get_config("llama3-8b", num_layers=2)
    model = build_model(cfg, device=gpu, seed=7)
    prompts = [torch.randint(1000, 100000, (48,)).tolist() for _ in range(batch)]
    outs = {}
    for on in (False, True):
        monkeypatch.setattr(ops, "GEMV_CHAIN", on)
        assert model._chain_ok(batch) == on
        ops._GEMM_USED.clear()  # before the engine: its graph captures run the decode forwards
        eng = Engine(model, EngineConfig(max_num_seqs=batch, max_num_batched_tokens=512, max_model_len=128,
                                         num_kv_blocks=batch * 8 + 1, use_graphs=True))
        outs[on] = eng.generate(prompts, SamplingParams(max_tokens=6, ignore_eos=True))
        small = set(k[3] for k in ops._GEMM_USED if k[0] <= 64)
        assert (ops.EPI_ADD_SS in small) == on, small
    for on in (False, True):
        for p, o in zip(prompts, outs[on]):
            toks = list(p)
            for t in o:
                lg = dense_logits(model, toks)[-1]
                best = int(lg.argmax())
                assert t == best or float(lg[best] - lg[t]) < 0.1 * float(lg.std()), (on, len(toks), best, t)
                toks.append(t)


def test_gemm_res_ss_odd_group_count(gpu, w4):
    """N = 3840 = 256 mod 512: the band ticket's row sum reads 30 groups of 128 columns (7
    16-byte loads + one 8-byte tail).  A 4-wide-only loop would add the next row's first two
    partials into every total."""
    M, N, K = 2048, 3840, 4096
    assert torch.ops.mlop.w4_chain_ok(M, N, K)
    torch.manual_seed(7)
    a = torch.randn(M, K, device=gpu, dtype=bf)
    w = (0.02 * torch.randn(N, K, device=gpu)).to(bf)
    r = torch.randn(M, N, device=gpu, dtype=bf)
    ss = ops.ss_buffer(M, N, gpu).fill_(float("nan"))
    ops.gemm_res_ss(a, w, r, ss)
    part, tot = ops.ss_parts(ss, M, N)
    close(part, r.float().pow(2).view(M, N // 128, 128).sum(-1), atol=1e-3, rtol=1e-4)
    close(tot, r.float().pow(2).sum(-1), atol=1e-2, rtol=1e-4)


def test_checkpoint_norms_folded_chain_matches_hf(gpu, w4, tmp_path, monkeypatch):
    """A checkpoint with trained (non-unit) RMSNorm weights: load_pretrained folds them into
    QKV / gate_up, so the 2048-row prefill runs the norm chain, and its first tokens are the
    fp32 transformers model's argmax (up to bf16 near-ties).  fold_norms=False keeps the norm
    weights and the chain off."""
    transformers = pytest.importorskip("transformers")
    from mlopamd.models import loader
    from mlopamd.runtime.engine import Engine, EngineConfig
    from mlopamd.runtime.sampler import SamplingParams

    torch.manual_seed(5)
    hf = transformers.LlamaForCausalLM(transformers.LlamaConfig(
        vocab_size=1024, hidden_size=H, intermediate_size=I, num_hidden_layers=1, num_attention_heads=32,
        num_key_value_heads=8, head_dim=128, max_position_embeddings=1024,
        rope_parameters={"rope_theta": 500000.0, "rope_type": "default"})).eval()
    with torch.no_grad():
        for layer in hf.model.layers:
            layer.input_layernorm.weight.uniform_(0.5, 1.5)
            layer.post_attention_layernorm.weight.uniform_(0.5, 1.5)
    hf.save_pretrained(tmp_path)
    assert not loader.load_pretrained(tmp_path, device=gpu, fold_norms=False).unit_norms
    model = loader.load_pretrained(tmp_path, device=gpu)
    assert model.unit_norms and model._chain_ok(2048)
    eng = Engine(model, EngineConfig(max_num_seqs=8, max_num_batched_tokens=2048, max_model_len=512,
                                     num_kv_blocks=8 * 32 + 1, use_graphs=False))
    g = torch.Generator().manual_seed(11)
    prompts = [torch.randint(3, 1000, (256,), generator=g).tolist() for _ in range(8)]
    ops._GEMM_USED.clear()
    outs = eng.generate(prompts, SamplingParams(max_tokens=1, ignore_eos=True))
    assert ops.EPI_ADD_SS in set(k[3] for k in ops._GEMM_USED)
    hf = hf.to(gpu)
    with torch.no_grad():
        lg = hf(torch.tensor(prompts, device=gpu)).logits[:, -1].float()
    for row, o in zip(lg, outs):
        assert row[o[0]] >= row.max() - 0.05 * row.abs().max(), (int(row.argmax()), o[0])
