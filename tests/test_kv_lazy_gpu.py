"""Lazily backed KV arena (ops/csrc/vmm.hip + runtime/kv_cache.py) on the GPU: the
first chunk is backed before the engine is ready, the rest on a native worker thread;
pages of later chunks arrive zeroed; an engine whose allocator grows mid-run produces
the same greedy tokens as one on an eagerly allocated cache; arenas return their memory."""
import time

import pytest
import torch

from mlopamd.models import build_model
from mlopamd.models.config import TINY_LLAMA
from mlopamd.runtime import kv_cache
from mlopamd.runtime.engine import Engine, EngineConfig
from mlopamd.runtime.sampler import SamplingParams

pytestmark = pytest.mark.gpu


@pytest.fixture
def small_chunks(monkeypatch):
    gran = int(torch.ops.mlop.vmm_granularity(0))
    chunk = max(gran, 64 << 10)  # 16 pages of a 1-kv-head, d=128 layer: many chunks
    monkeypatch.setattr(kv_cache, "CHUNK_BYTES_PER_REGION", chunk)
    monkeypatch.setattr(kv_cache, "INITIAL_BYTES", 1)  # back only the first chunk up front
    return chunk


def _wait_ready(kv, timeout=30.0):
    t0 = time.time()
    while kv.ready_blocks() < kv.num_blocks:
        assert time.time() - t0 < timeout, f"background fill stuck at {kv.ready_blocks()}/{kv.num_blocks}"
        time.sleep(0.01)


def test_vmm_supported(gpu):
    assert torch.ops.mlop.vmm_supported(0), "HIP VMM must be available: the lazy KV path is the default"
    assert torch.ops.mlop.vmm_granularity(0) > 0


def test_lazy_kv_fill_and_zero(gpu, small_chunks):
    kv = kv_cache.KVCache(2, 2048, 1, 128, gpu, torch.bfloat16, lazy=True)
    assert kv.lazy and kv.n_chunks >= 4
    assert kv.ready_blocks() == kv.chunk_blocks  # only the first chunk before the fill starts
    assert kv.chunk_blocks * 128 * 16 * 2 == small_chunks
    kv.k[0][1].fill_(3.0)                         # the backed chunk is usable right away
    assert float(kv.k[0][1].float().sum()) == 3.0 * 16 * 128
    kv.start_background_fill()
    _wait_ready(kv)
    for t in (kv.k[1], kv.v[1], kv.k[0]):
        assert int(t[-1].abs().sum().item()) == 0   # last page of the last chunk: backed and zeroed
    kv.v[1][-1].fill_(-2.0)
    torch.cuda.synchronize()
    assert float(kv.v[1][-1].float().mean()) == -2.0
    assert float(kv.v[0][-1].float().abs().sum()) == 0.0  # regions do not alias


def test_lazy_arena_releases_memory(gpu):
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    for _ in range(3):
        kv = kv_cache.KVCache(8, 40000, 8, 128, gpu, torch.bfloat16, lazy=True)  # ~21 GB
        kv.start_background_fill()
        _wait_ready(kv, 120.0)
        assert torch.cuda.mem_get_info()[0] < free0 - 15e9
        del kv
        torch.cuda.synchronize()
    assert torch.cuda.mem_get_info()[0] > free0 - 2e9


def test_engine_grows_kv_mid_run(gpu, small_chunks, monkeypatch):
    """Greedy tokens on a lazily backed cache whose allocator grows while requests run
    equal those of the same model on an eager cache."""
    model = build_model(TINY_LLAMA, device=gpu, seed=5)
    prompts = [torch.randint(2, 500, (200 + 10 * i,), generator=torch.Generator().manual_seed(i)).tolist()
               for i in range(24)]
    outs = {}
    from mlopamd.runtime import kv_cache

    for lazy in ("1", "0"):
        monkeypatch.setattr(kv_cache, "LAZY", lazy == "1")
        eng = Engine(model, EngineConfig(max_num_seqs=24, max_num_batched_tokens=2048, max_model_len=512,
                                         num_kv_blocks=2048, use_graphs=True, graph_buckets=(1, 8, 24)))
        assert eng.kv.lazy == (lazy == "1")
        if eng.kv.lazy:
            assert eng.stats["kv_ready_blocks_at_start"] < 2048
        outs[lazy] = eng.generate(prompts, SamplingParams(max_tokens=24, ignore_eos=True))
        if eng.kv.lazy:
            _wait_ready(eng.kv)
            eng.step()  # an idle step picks up the remaining chunks
            assert eng.alloc.available == 2048
        del eng
    assert outs["1"] == outs["0"]
