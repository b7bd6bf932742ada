"""Engine logic on CPU (reference ops): paging, chunked prefill, preemption,
row/slot bookkeeping — checked against the dense recompute oracle."""
import numpy as np
import pytest
import torch

from mlopamd import ops
from mlopamd.models import build_model
from mlopamd.models.config import TINY_LLAMA, TINY_MIXTRAL
from mlopamd.models.reference import dense_logits
from mlopamd.runtime.attn_meta import plan_partitions
from mlopamd.runtime.engine import Engine, EngineConfig, Status
from mlopamd.runtime.kv_cache import BlockAllocator
from mlopamd.runtime.sampler import SamplingParams, sample_reference


def greedy_ref(model, prompt, n):
    toks = list(prompt)
    out = []
    for _ in range(n):
        t = int(dense_logits(model, toks)[-1].argmax())
        out.append(t)
        toks.append(t)
    return out


@pytest.fixture(scope="module")
def tiny():
    torch.manual_seed(0)
    return build_model(TINY_LLAMA, device="cpu", dtype=torch.float32, seed=1)


def test_generate_matches_dense_with_chunking(tiny):
    eng = Engine(tiny, EngineConfig(max_num_seqs=8, max_num_batched_tokens=40, max_model_len=256,
                                    num_kv_blocks=64, use_graphs=False))
    prompts = [torch.randint(2, 500, (n,)).tolist() for n in (5, 33, 17, 70)]
    outs = eng.generate(prompts, SamplingParams(max_tokens=6, ignore_eos=True))
    for p, o in zip(prompts, outs):
        assert o == greedy_ref(tiny, p, 6)
    assert eng.stats["prefill_steps"] >= 3  # the 70-token prompt needed chunks
    assert eng.alloc.num_free == eng.alloc.num_blocks - 1  # everything released


@pytest.mark.parametrize("mixed", [True, False])
def test_mixed_prefill_decode_steps(tiny, mixed):
    """Requests arriving while others decode: with mixing, their prompt chunks
    ride in the decode step (one ragged forward); outputs stay exact."""
    eng = Engine(tiny, EngineConfig(max_num_seqs=8, max_num_batched_tokens=48, max_model_len=256,
                                    num_kv_blocks=96, use_graphs=False, mixed_prefill=mixed,
                                    mixed_min_chunk=8))
    prompts = [torch.randint(2, 500, (n,)).tolist() for n in (7, 40, 12, 65, 3)]
    seqs = [eng.add_request(prompts[0], SamplingParams(max_tokens=12, ignore_eos=True))]
    for p in prompts[1:]:
        eng.step()
        eng.step()
        seqs.append(eng.add_request(p, SamplingParams(max_tokens=12, ignore_eos=True)))
    while eng.has_work():
        eng.step()
    for p, s in zip(prompts, seqs):
        assert s.output == greedy_ref(tiny, p, 12)
    assert (eng.stats["mixed_steps"] > 0) == mixed
    assert eng.alloc.num_free == eng.alloc.num_blocks - 1


def test_mixed_step_sampling_params(tiny):
    """A mixed step with non-greedy decode rows and a greedy prefill completes
    through the general sampler path."""
    eng = Engine(tiny, EngineConfig(max_num_seqs=4, max_num_batched_tokens=64, max_model_len=128,
                                    num_kv_blocks=48, use_graphs=False, mixed_min_chunk=8))
    a = eng.add_request([5, 6, 7, 8], SamplingParams(max_tokens=6, temperature=0.8, top_k=5, ignore_eos=True))
    eng.step()
    b = eng.add_request(list(range(10, 30)), SamplingParams(max_tokens=4, ignore_eos=True))
    while eng.has_work():
        eng.step()
    assert eng.stats["mixed_steps"] >= 1
    assert len(a.output) == 6 and b.output == greedy_ref(tiny, list(range(10, 30)), 4)


def test_preemption_recompute(tiny):
    # 12 usable pages: two 60-token sequences cannot both grow to 100 tokens
    eng = Engine(tiny, EngineConfig(max_num_seqs=4, max_num_batched_tokens=256, max_model_len=256,
                                    num_kv_blocks=13, use_graphs=False))
    prompts = [torch.randint(2, 500, (60,)).tolist() for _ in range(2)]
    outs = eng.generate(prompts, SamplingParams(max_tokens=40, ignore_eos=True))
    assert eng.stats["preemptions"] >= 1
    for p, o in zip(prompts, outs):
        assert o[:8] == greedy_ref(tiny, p, 8)
        assert len(o) == 40


def test_stop_conditions(tiny):
    eng = Engine(tiny, EngineConfig(max_num_seqs=2, max_model_len=64, num_kv_blocks=16, use_graphs=False))
    s = eng.add_request([3, 4, 5], SamplingParams(max_tokens=1000, ignore_eos=True))
    while eng.has_work():
        eng.step()
    assert s.status == Status.FINISHED and s.finish_reason == "length" and s.length == 64
    # eos stop: force eos = the greedy next token
    first = greedy_ref(tiny, [7, 8, 9], 1)[0]
    s2 = eng.add_request([7, 8, 9], SamplingParams(max_tokens=10, stop_token_ids=[first]))
    while eng.has_work():
        eng.step()
    assert s2.finish_reason == "stop" and s2.output == [first]


def test_abort_releases(tiny):
    eng = Engine(tiny, EngineConfig(max_num_seqs=2, max_model_len=64, num_kv_blocks=16, use_graphs=False))
    s = eng.add_request(list(range(2, 30)), SamplingParams(max_tokens=20))
    eng.step()
    eng.abort(s.seq_id)
    assert s.finish_reason == "abort" and eng.alloc.num_free == 15 and not eng.has_work()


def test_mixtral_cpu_matches_dense():
    torch.manual_seed(0)
    m = build_model(TINY_MIXTRAL, device="cpu", dtype=torch.float32, seed=2)
    eng = Engine(m, EngineConfig(max_num_seqs=4, max_num_batched_tokens=64, max_model_len=128,
                                 num_kv_blocks=32, use_graphs=False))
    prompts = [torch.randint(2, 500, (n,)).tolist() for n in (9, 20)]
    outs = eng.generate(prompts, SamplingParams(max_tokens=4, ignore_eos=True))
    for p, o in zip(prompts, outs):
        assert o == greedy_ref(m, p, 4)


def test_block_allocator():
    a = BlockAllocator(10)
    x = a.allocate(4)
    assert 0 not in x and len(set(x)) == 4 and a.num_free == 5
    with pytest.raises(MemoryError):
        a.allocate(6)
    a.free(x)
    assert a.num_free == 9 and a.usage() == 0.0


@pytest.mark.parametrize("tiles,nkv,ctx", [(256, 8, 2048), (1, 8, 4096), (4, 1, 300), (64, 8, 100)])
def test_plan_partitions_covers_context(tiles, nkv, ctx):
    part, n = plan_partitions(tiles, nkv, ctx)
    assert part % 32 == 0 and part * n >= ctx and part * (n - 1) < ctx


def test_sampler_reference_semantics():
    torch.manual_seed(0)
    x = torch.randn(4, 100)
    t = torch.tensor([0.0, 1.0, 1.0, 1.0])
    k = torch.tensor([0, 1, 5, 0], dtype=torch.int32)
    p = torch.tensor([1.0, 1.0, 1.0, 0.3])
    u = torch.tensor([0.5, 0.99, 0.0, 0.999])
    out = sample_reference(x, t, k, p, u)
    am = x.argmax(-1)
    assert out[0] == am[0] and out[1] == am[1] and out[2] == am[2]
    assert int(out[3]) in torch.topk(x[3], 100).indices[:20].tolist()


def test_moe_reference_ops_roundtrip():
    torch.manual_seed(0)
    T, H, E, k = 13, 32, 4, 2
    x = torch.randn(T, H)
    w, idx = ops.moe_route(torch.randn(T, E), k)
    xp, off, src, inv = ops.moe_permute(x, idx, 0, E)
    n = int(off[-1])
    assert n == T * k
    # identity experts: combine must give sum_j w_j * x = x (weights renormalised)
    y = xp.clone()
    torch.testing.assert_close(ops.moe_combine(y, inv, w), x, atol=1e-5, rtol=1e-5)
    # a partial expert range (EP shard) only covers its slots
    xp2, off2, src2, inv2 = ops.moe_permute(x, idx, 2, 2)
    assert int(off2[-1]) == int(((idx >= 2)).sum())
    assert int((inv2 >= 0).sum()) == int(off2[-1])


def test_block_allocator_grow():
    """Lazily backed KV: only ids below ``available`` are handed out until grow()."""
    a = BlockAllocator(100, available=10)
    assert a.num_free == 9 and a.usage() == 0.0
    x = a.allocate(9)
    assert max(x) < 10 and not a.can_allocate(1)
    assert a.grow(40) == 30 and a.available == 40 and a.num_free == 30
    y = a.allocate(30)
    assert set(y) == set(range(10, 40))
    assert a.grow(5) == 0 and a.grow(1000) == 60 and a.available == 100
    a.free(x + y)
    assert a.num_free == 99 and a.usage() == 0.0


def test_allocator_prefix_cache_lru():
    a = BlockAllocator(8)
    x = a.allocate(3)
    for b, h in zip(x, (11, 22, 33)):
        a.register(b, h)
    assert a.num_cached == 3 and a.lookup(22) == x[1]
    a.free(x)  # cached pages stay cached while free
    assert a.num_free == 7 and a.num_cached == 3
    a.take(x[0])  # a prefix hit on a free cached page
    assert a.num_free == 6
    y = a.allocate(4)  # uncached pages first, no eviction
    assert not set(y) & set(x) and a.num_cached == 3
    z = a.allocate(1)  # then the least recently freed cached page is evicted
    assert z[0] in x[1:] and a.num_cached == 2 and a.lookup(22 if z[0] == x[1] else 33) is None
    with pytest.raises(MemoryError):
        a.allocate(2)
    a.free([x[0]])
    assert a.num_free == 2


def _shared_prefix_prompts(n, prefix_len=70, seed=3):
    g = torch.Generator().manual_seed(seed)
    prefix = torch.randint(2, 500, (prefix_len,), generator=g).tolist()
    return [prefix + torch.randint(2, 500, (5 + 7 * i,), generator=g).tolist() for i in range(n)]


@pytest.mark.parametrize("mixed", [True, False])
def test_prefix_caching_matches_uncached(mixed):
    """Requests sharing a 70-token prefix: with the prefix cache the later ones skip the
    shared pages' prefill (hits counted), and every greedy output equals the
    no-cache engine's (and the dense oracle's)."""
    m = build_model(TINY_LLAMA, device="cpu", dtype=torch.float32, seed=4)
    prompts = _shared_prefix_prompts(6)
    outs = {}
    for cache in (True, False):
        eng = Engine(m, EngineConfig(max_num_seqs=4, max_num_batched_tokens=96, max_model_len=256, num_kv_blocks=64,
                                     use_graphs=False, enable_prefix_caching=cache, mixed_prefill=mixed))
        first = eng.generate(prompts[:1], SamplingParams(max_tokens=5, ignore_eos=True))
        rest = eng.generate(prompts[1:], SamplingParams(max_tokens=5, ignore_eos=True))
        outs[cache] = first + rest
        if cache:
            assert eng.stats["prefix_hit_tokens"] >= 5 * 64  # 4 full shared pages per later request
        else:
            assert eng.stats["prefix_hit_tokens"] == 0
    assert outs[True] == outs[False]
    for p, o in zip(prompts[:2], outs[True][:2]):
        assert o == greedy_ref(m, p, 5)


def test_prefix_cache_survives_preemption():
    """A tiny KV pool forces preemptions; re-admitted sequences re-match their own cached
    pages and the outputs still equal the dense oracle."""
    m = build_model(TINY_LLAMA, device="cpu", dtype=torch.float32, seed=6)
    prompts = _shared_prefix_prompts(5, prefix_len=40, seed=9)
    eng = Engine(m, EngineConfig(max_num_seqs=5, max_num_batched_tokens=64, max_model_len=256, num_kv_blocks=13,
                                 use_graphs=False))
    outs = eng.generate(prompts, SamplingParams(max_tokens=40, ignore_eos=True))
    assert eng.stats["preemptions"] > 0 and eng.stats["prefix_hit_tokens"] > 0
    for p, o in zip(prompts, outs):
        assert o == greedy_ref(m, p, 40)
    assert eng.alloc.num_free == eng.alloc.available - 1  # every reference returned


@pytest.mark.parametrize("mixed", [True, False])
def test_running_rows_bookkeeping_randomized(tiny, mixed):
    """The decode hot path keeps ``running``'s rows / output lists in step incrementally
    (appends, masked finishes, preemption pops; aborts force a rebuild).  Under random
    arrivals, aborts, stop tokens and a KV pool small enough to preempt, after every step
    the incremental state must equal a rebuild, and every sequence that ran to completion
    must still match the dense greedy oracle."""
    rng = np.random.default_rng(7)
    eng = Engine(tiny, EngineConfig(max_num_seqs=6, max_num_batched_tokens=48, max_model_len=256,
                                    num_kv_blocks=12, use_graphs=False, mixed_prefill=mixed,
                                    mixed_min_chunk=8, enable_prefix_caching=False))
    seqs = []
    for it in range(160):
        if rng.random() < 0.35 and len(seqs) < 24:
            p = rng.integers(2, 500, size=int(rng.integers(3, 40))).tolist()
            stop = [int(rng.integers(2, 500))] if rng.random() < 0.3 else []
            seqs.append(eng.add_request(p, SamplingParams(max_tokens=int(rng.integers(2, 40)), ignore_eos=True,
                                                          stop_token_ids=stop)))
        if rng.random() < 0.04:
            live = [s for s in seqs if s.status != Status.FINISHED]
            if live:
                eng.abort(live[int(rng.integers(len(live)))].seq_id)
        if eng.has_work():
            eng.step()
        rows = eng._sync_rows()
        assert rows.tolist() == [s.row for s in eng.running]
        assert len(eng._outs) == len(eng.running)
        assert all(o is s.output for o, s in zip(eng._outs, eng.running))
    while eng.has_work():
        eng.step()
    assert eng.stats["preemptions"] > 0
    done = [s for s in seqs if s.finish_reason in ("length", "stop")]
    assert len(done) >= 8
    for s in done[:8]:
        ref = greedy_ref(tiny, s.prompt, len(s.output))
        assert s.output == ref
    assert eng.alloc.num_free == eng.alloc.num_blocks - 1


def test_prefix_keys_are_cryptographic_digests():
    """Page keys are chained BLAKE2b digests of the token ids (not Python hash()): different
    pages never share a key in practice, equal prefixes always do, and the chain makes a
    page's key depend on every earlier token."""
    from mlopamd.runtime.kv_cache import BLOCK_SIZE, prefix_hashes

    a = list(range(3 * BLOCK_SIZE))
    b = list(a)
    b[1] = 10**9  # differs in page 0 only
    ha, hb = prefix_hashes(a, 3), prefix_hashes(b, 3)
    assert all(isinstance(h, bytes) and len(h) == 16 for h in ha)
    assert all(x != y for x, y in zip(ha, hb))  # the chain carries page 0's difference forward
    assert prefix_hashes(a, 3) == ha and prefix_hashes(a, 3, start=1, prev=ha[0]) == ha[1:]
    # Python's tuple hash of small ints collides for these (-1 and -2 hash alike); the digest does not
    c, d = [-1] * BLOCK_SIZE, [-2] * BLOCK_SIZE
    assert hash(tuple(c)) == hash(tuple(d)) and prefix_hashes(c, 1) != prefix_hashes(d, 1)


def test_kv_background_fill_failure_keeps_serving(tiny):
    """A lazily backed KV arena whose background fill fails (another process took the memory)
    stops growing; the engine keeps serving from the pages already backed and records it."""
    eng = Engine(tiny, EngineConfig(max_num_seqs=4, max_num_batched_tokens=64, max_model_len=256,
                                    num_kv_blocks=64, use_graphs=False))
    eng.alloc = BlockAllocator(64, available=24)  # only 24 pages backed so far
    calls = {"n": 0}

    def ready_blocks():
        calls["n"] += 1
        eng.kv.fill_failed = True  # the native worker reported an out-of-memory chunk
        return 32  # chunks backed before the failure stay usable

    eng.kv.ready_blocks = ready_blocks
    outs = eng.generate([[5, 6, 7, 8], list(range(20, 60))], SamplingParams(max_tokens=8, ignore_eos=True))
    assert [len(o) for o in outs] == [8, 8]
    assert eng.stats["kv_fill_failed"] == 1 and eng.alloc.available == 32 and calls["n"] == 1
    assert outs[0] == greedy_ref(tiny, [5, 6, 7, 8], 8)


def test_multiple_eos_ids_stop_generation(tiny):
    """HF eos_token_id lists (Llama-3.1-Instruct: <|end_of_text|>, <|eom_id|>, <|eot_id|>) all stop."""
    import dataclasses

    prompt = [5, 9, 11]
    free = greedy_ref(tiny, prompt, 6)
    m = build_model(dataclasses.replace(TINY_LLAMA, eos_token_id=499, extra_eos_ids=(free[2],)), device="cpu",
                    dtype=torch.float32, seed=1)
    eng = Engine(m, EngineConfig(max_num_seqs=2, max_num_batched_tokens=32, max_model_len=128, num_kv_blocks=32,
                                 use_graphs=False))
    (out,) = eng.generate([prompt], SamplingParams(max_tokens=6))
    assert out == free[:3]


@pytest.mark.parametrize("graphs_like_bucket", [False, True])
def test_async_scheduling_matches_sync(tiny, graphs_like_bucket):
    """One-step-ahead scheduling (step t+1 launched before step t's tokens are applied; decode
    ids gathered on the device from the in-flight step; EOS / stop-token rows decoded once
    more and their stale result dropped; aborts and preemption mid-flight) produces exactly
    the synchronous engine's outputs and finish reasons."""
    rng = np.random.default_rng(11)
    prompts = [rng.integers(2, 500, size=int(rng.integers(3, 50))).tolist() for _ in range(14)]
    # stop tokens that will actually fire: each odd request stops at its own 3rd greedy token
    probe = Engine(tiny, EngineConfig(max_num_seqs=8, max_model_len=256, num_kv_blocks=64, use_graphs=False,
                                      async_scheduling=False))
    third = probe.generate(prompts, SamplingParams(max_tokens=3, ignore_eos=True))
    params = [SamplingParams(max_tokens=int(4 + i % 9), ignore_eos=True,
                             stop_token_ids=[third[i][2]] if i % 2 else []) for i in range(len(prompts))]

    def run(asy):
        eng = Engine(tiny, EngineConfig(max_num_seqs=5, max_num_batched_tokens=40, max_model_len=256,
                                        num_kv_blocks=14, use_graphs=False, mixed_min_chunk=8,
                                        async_scheduling=asy, prefill_min_batch=1 if graphs_like_bucket else 2))
        seqs, i, it = [], 0, 0
        while i < len(prompts) or eng.has_work():
            if i < len(prompts) and it % 2 == 0:
                seqs.append(eng.add_request(prompts[i], params[i]))
                i += 1
            if it == 12:
                eng.abort(seqs[-1].seq_id)  # just admitted: prefilling or with a token in flight
            eng.step()
            it += 1
        assert eng.alloc.num_free == eng.alloc.available - 1
        return [(s.output, s.finish_reason) for s in seqs], eng.stats

    sync, _ = run(False)
    asy, st = run(True)
    assert st["async_host_us"] > 0
    assert asy == sync
    assert any(r == "stop" for _, r in asy) and any(r == "abort" for _, r in asy)


def test_dead_peer_error_word_fails_the_step():
    """A device-side collective whose flag wait timed out (a peer rank died or wedged) reports it
    in its host-mapped error word; the engine checks it after every step and raises instead of
    serving the garbage results (the launcher then restarts the predictor)."""
    model = build_model(TINY_LLAMA, device="cpu", dtype=torch.float32, seed=1)
    eng = Engine(model, EngineConfig(max_num_seqs=4, max_model_len=128, num_kv_blocks=32, use_graphs=False))

    class _Car:
        code = 0

        def error(self):
            return self.code

    car = _Car()
    model.ps.tp.car = car
    try:
        eng.add_request([5, 6, 7], SamplingParams(max_tokens=4, ignore_eos=True))
        eng.step()  # healthy
        car.code = 1
        with pytest.raises(RuntimeError, match="peer flag wait timed out"):
            eng.step()
    finally:
        model.ps.tp.car = None
