"""End-to-end GPU checks: the engine (HIP kernels, paging, chunked prefill,
hipGraph decode) against the dense fp32 recompute oracle."""
import pytest
import torch

from mlopamd.models import build_model
from mlopamd.models.config import TINY_LLAMA, TINY_MIXTRAL, get_config
from mlopamd.models.reference import dense_logits
from mlopamd.runtime.engine import Engine, EngineConfig
from mlopamd.runtime.sampler import SamplingParams

pytestmark = pytest.mark.gpu


def _check_greedy(model, prompts, outs, tol=0.05):
    for p, o in zip(prompts, outs):
        toks = list(p)
        for t in o:
            lg = dense_logits(model, toks)[-1]
            best = int(lg.argmax())
            gap = float(lg[best] - lg[t])
            assert t == best or gap < tol * float(lg.std()), (len(toks), best, t, gap)
            toks.append(t)


@pytest.mark.parametrize("graphs", [False, True])
@pytest.mark.parametrize("cfg", [TINY_LLAMA, TINY_MIXTRAL], ids=["llama", "mixtral"])
def test_engine_matches_dense(gpu, graphs, cfg):
    torch.manual_seed(0)
    model = build_model(cfg, device=gpu, seed=3)
    eng = Engine(model, EngineConfig(max_num_seqs=8, max_num_batched_tokens=64, max_model_len=512,
                                     num_kv_blocks=128, use_graphs=graphs, graph_buckets=(1, 2, 4, 8)))
    prompts = [torch.randint(2, 500, (n,)).tolist() for n in (5, 40, 17, 130, 3)]
    outs = eng.generate(prompts, SamplingParams(max_tokens=10, ignore_eos=True))
    if graphs:
        assert eng.stats["graph_steps"] > 0
    _check_greedy(model, prompts, outs)


def test_llama3_8b_layer_shapes_decode(gpu):
    """Full Llama-3-8B width (2 layers) through graphs at batch 64: shapes the bench uses."""
    cfg = get_config("llama3-8b", num_layers=2)
    model = build_model(cfg, device=gpu)
    eng = Engine(model, EngineConfig(max_num_seqs=64, max_num_batched_tokens=2048, max_model_len=1024,
                                     num_kv_blocks=64 * 64 + 1, graph_buckets=(1, 8, 64)))
    prompts = [torch.randint(1000, 100000, (100 + 7 * i,)).tolist() for i in range(64)]
    outs = eng.generate(prompts, SamplingParams(max_tokens=4, ignore_eos=True))
    assert all(len(o) == 4 for o in outs)
    assert eng.stats["graph_steps"] >= 3
    _check_greedy(model, prompts[:3], [o[:2] for o in outs[:3]], tol=0.1)


@pytest.mark.parametrize("mixed", [True, False])
def test_engine_staggered_arrivals(gpu, mixed):
    """Requests arriving while others decode (the serving pattern): with mixing
    their prompt chunks share the decode step's forward (ragged attention over
    decode + prefill tiles); greedy outputs match the dense oracle either way."""
    torch.manual_seed(0)
    model = build_model(TINY_LLAMA, device=gpu, seed=5)
    eng = Engine(model, EngineConfig(max_num_seqs=8, max_num_batched_tokens=96, max_model_len=512,
                                     num_kv_blocks=128, graph_buckets=(1, 2, 4, 8), mixed_prefill=mixed,
                                     mixed_min_chunk=8))
    prompts = [torch.randint(2, 500, (n,)).tolist() for n in (9, 70, 21, 150, 4, 33)]
    seqs = [eng.add_request(prompts[0], SamplingParams(max_tokens=12, ignore_eos=True))]
    for p in prompts[1:]:
        eng.step()
        seqs.append(eng.add_request(p, SamplingParams(max_tokens=12, ignore_eos=True)))
    while eng.has_work():
        eng.step()
    assert (eng.stats["mixed_steps"] > 0) == mixed
    _check_greedy(model, prompts, [s.output for s in seqs])


@pytest.mark.parametrize("cfg", [TINY_LLAMA, TINY_MIXTRAL], ids=["llama", "mixtral"])
def test_prefix_caching_gpu(gpu, cfg):
    """Requests sharing a 100-token prefix on the GPU engine (graphs, mixed steps): the
    later ones reuse the cached pages (hits counted) and still decode the dense oracle's
    greedy tokens."""
    torch.manual_seed(0)
    model = build_model(cfg, device=gpu, seed=7)
    g = torch.Generator().manual_seed(1)
    prefix = torch.randint(2, 500, (100,), generator=g).tolist()
    prompts = [prefix + torch.randint(2, 500, (3 + 11 * i,), generator=g).tolist() for i in range(5)]
    eng = Engine(model, EngineConfig(max_num_seqs=8, max_num_batched_tokens=128, max_model_len=512,
                                     num_kv_blocks=128, graph_buckets=(1, 2, 4, 8)))
    outs = eng.generate(prompts[:1], SamplingParams(max_tokens=8, ignore_eos=True))
    outs += eng.generate(prompts[1:], SamplingParams(max_tokens=8, ignore_eos=True))
    assert eng.stats["prefix_hit_tokens"] >= 4 * 96  # 6 full shared pages per later request
    _check_greedy(model, prompts, outs)


def test_mixtral_decode_fused_moe_glue(gpu):
    """hidden 1024: the decode steps take the one-launch MoE dispatch (router GEMV + route +
    sort + gather) and the combine fused into the residual add + RMSNorm; greedy tokens
    still follow the dense oracle."""
    from dataclasses import replace

    cfg = replace(TINY_MIXTRAL, hidden_size=1024, intermediate_size=512)
    torch.manual_seed(0)
    model = build_model(cfg, device=gpu, seed=4)
    x = torch.randn(3, 1024, device=gpu, dtype=torch.bfloat16)
    from mlopamd import ops

    assert ops.moe_dispatch_small(x, model.layers[0]["router"], 2, 0, cfg.num_experts) is not None
    eng = Engine(model, EngineConfig(max_num_seqs=4, max_num_batched_tokens=64, max_model_len=512,
                                     num_kv_blocks=64, graph_buckets=(1, 2, 4)))
    prompts = [torch.randint(2, 500, (n,)).tolist() for n in (5, 33, 70)]
    outs = eng.generate(prompts, SamplingParams(max_tokens=8, ignore_eos=True))
    assert eng.stats["graph_steps"] > 0
    _check_greedy(model, prompts, outs)


@pytest.mark.parametrize("graphs,async_reduce", [(False, False), (True, False), (True, True)])
def test_kernel_time_sampler_on_engine_steps(gpu, graphs, async_reduce):
    """G3: the in-process sampler (runtime/gpu_metrics.KernelTimeSampler, what the predictor
    exports as mlop_kernel_time_fraction) sees this engine's HIP kernels -- eager launches and
    decode-graph replays -- and splits them into the classes the canary gate guards.
    ``async_reduce``: the event reduction runs on a helper thread (the predictor's default)."""
    from mlopamd.runtime.gpu_metrics import KernelTimeSampler

    model = build_model(TINY_LLAMA, device=gpu, seed=3)
    eng = Engine(model, EngineConfig(max_num_seqs=8, max_num_batched_tokens=64, max_model_len=512,
                                     num_kv_blocks=128, use_graphs=graphs, graph_buckets=(1, 2, 4, 8)))
    for p in (torch.randint(2, 500, (n,)).tolist() for n in (5, 40, 17)):
        eng.add_request(p, SamplingParams(max_tokens=12, ignore_eos=True))
    for _ in range(3):  # past the prefill: the sampled step is a decode step
        eng.step()
    got = []
    s = KernelTimeSampler(period_s=1e-6, on_shares=got.append, async_reduce=async_reduce)
    s.warm()
    s.before_step(0.0)  # the first call only arms the first window, one period later
    assert s._prof is None
    s.before_step(1.0)
    eng.step()
    assert s.after_step(1.0) is None  # never waits for the device: the window stays open
    sh = None
    for k in range(50):  # closes at the first step boundary after the profiled step completed
        eng.step()
        sh = s.after_step(2.0 + k)
        if s.windows:
            break
    if async_reduce:  # reduced on the helper thread: published once it finished
        assert sh is None
        s.join()
        sh = s.last
    assert got and sh == got[0] and s.windows == 1, sh
    assert s.host_ms and s.warm_ms is not None
    assert abs(sum(sh.values()) - 1.0) < 1e-6
    assert sh.get("gemm", 0) > 0 and sh.get("attention", 0) > 0, sh
