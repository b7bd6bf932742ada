"""Multi-process (gloo, world_size 2) tests of the parallel paths on CPU:
TP lock-step engine == TP=1 engine (Llama and Mixtral TP+EP), expert-parallel
all-to-all MoE == single-rank MoE, process-group helpers."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, world, port, fn_name, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = globals()[fn_name](rank, world)
        torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def run_ranks(fn_name, world=2):
    d = tempfile.mkdtemp()
    mp.start_processes(_entry, args=(world, _free_port(), fn_name, d), nprocs=world, join=True,
                       start_method="spawn")
    return [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=False) for r in range(world)]


PROMPTS = [[5, 9, 11, 40, 2, 7], list(range(20, 61)), [100, 3]]


def _tp_engine(cfg_name, world=2, **overrides):
    from mlopamd.models import build_model
    from mlopamd.models.config import get_config
    from mlopamd.parallel.comm import make_parallel_state
    from mlopamd.runtime.engine import Engine, EngineConfig
    from mlopamd.runtime.sampler import SamplingParams

    cfg = get_config(cfg_name, **overrides)
    full = build_model(cfg, device="cpu", dtype=torch.float32, seed=4)
    ps = make_parallel_state(tp_size=world, ep_size=world)
    shard = build_model(cfg, device="cpu", dtype=torch.float32, pstate=ps, seed=4).load_shard_from(full)
    ec = EngineConfig(max_num_seqs=4, max_num_batched_tokens=32, max_model_len=128, num_kv_blocks=40, use_graphs=False)
    eng = Engine(shard, ec)
    params = SamplingParams(max_tokens=6, ignore_eos=True)
    # a sampled request alongside greedy ones: the full-logits gather path
    sampled = [params] * (len(PROMPTS) - 1) + [SamplingParams(max_tokens=6, ignore_eos=True, temperature=0.8,
                                                              top_k=20)]
    if ps.tp_rank == 0:
        outs = eng.generate(PROMPTS, params)
        mixed = eng.generate(PROMPTS, sampled)
        stats = dict(eng.stats)
        eng.shutdown()
        ref_eng = Engine(full, ec)
        ref = ref_eng.generate(PROMPTS, params)
        ref_mixed = ref_eng.generate(PROMPTS, sampled)
        return {"tp": outs, "ref": ref, "mixed": mixed, "ref_mixed": ref_mixed, "stats": stats}
    eng.worker_loop()
    return {"worker_steps": eng.stats["worker_steps"]}


def tp_sync(rank, world):
    """Leader's sync_point() is a world barrier the parked TP worker joins."""
    from mlopamd.models import build_model
    from mlopamd.models.config import get_config
    from mlopamd.parallel.comm import make_parallel_state
    from mlopamd.runtime.engine import Engine, EngineConfig
    from mlopamd.runtime.sampler import SamplingParams

    ps = make_parallel_state(tp_size=2)
    m = build_model(get_config("tiny-llama"), device="cpu", dtype=torch.float32, pstate=ps, seed=4)
    eng = Engine(m, EngineConfig(max_num_seqs=2, max_num_batched_tokens=32, max_model_len=64, num_kv_blocks=16,
                                 use_graphs=False))
    if ps.tp_rank == 0:
        eng.sync_point()
        out = eng.generate([[5, 6, 7]], SamplingParams(max_tokens=3, ignore_eos=True))
        eng.sync_point()
        eng.shutdown()
        return {"out": out}
    eng.worker_loop()
    return {"worker_steps": eng.stats["worker_steps"]}


def test_tp_sync_point_barrier():
    r0, r1 = run_ranks("tp_sync")
    assert len(r0["out"][0]) == 3 and r1["worker_steps"] > 0


def tp_llama(rank, world):
    return _tp_engine("tiny-llama")


def tp_mixtral(rank, world):
    return _tp_engine("tiny-mixtral")


def tp4_llama(rank, world):
    return _tp_engine("tiny-llama", world)


def tp8_llama(rank, world):  # 8 q heads so TP=8 shards them; the single kv head is replicated
    return _tp_engine("tiny-llama", world, num_heads=8)


def tp4_mixtral(rank, world):
    return _tp_engine("tiny-mixtral", world)


@pytest.mark.parametrize("fn,world", [("tp_llama", 2), ("tp_mixtral", 2), ("tp4_llama", 4),
                                      ("tp8_llama", 8), ("tp4_mixtral", 4)])
def test_tp_engine_matches_tp1(fn, world):
    """TP=2/4/8 lock-step engine == TP=1 on the same weights: greedy tokens, and a batch with
    one sampled request (same seed: the full-logits gather path feeds the same sampler)."""
    res = run_ranks(fn, world)
    r0 = res[0]
    assert r0["tp"] == r0["ref"]
    assert r0["mixed"][:-1] == r0["ref_mixed"][:-1] and len(r0["mixed"][-1]) == 6
    assert r0["mixed"][-1] == r0["ref_mixed"][-1]
    # ONE metadata collective per step (packed header + metadata + ids)
    assert r0["stats"]["tp_sync_calls"] > 0
    assert all(r["worker_steps"] > 0 for r in res[1:])


def ep_alltoall(rank, world):
    from mlopamd import ops
    from mlopamd.parallel.comm import make_parallel_state
    from mlopamd.parallel.moe import local_experts, moe_forward

    torch.manual_seed(0)
    E, H, I, k = 4, 64, 32, 2
    router = torch.randn(E, H)
    w13 = 0.1 * torch.randn(E, 2 * I, H)
    w2 = 0.1 * torch.randn(E, H, I)
    xs = [torch.randn(7, H), torch.randn(5, H)]  # different token counts per rank
    ps = make_parallel_state(tp_size=1, ep_size=world)  # DP attention + EP MoE layout
    ep = ps.ep
    assert ps.tp.size == 1 and ep.size == world and ep.rank == rank
    nl = E // world
    out = moe_forward(xs[rank], router, w13[rank * nl:(rank + 1) * nl], w2[rank * nl:(rank + 1) * nl], k, ep,
                      rank * nl, nl, mode="alltoall", cap_tokens=max(x.shape[0] for x in xs))
    # single-rank reference with all experts
    topw, topi = ops.moe_route(torch.nn.functional.linear(xs[rank], router), k)
    ref = local_experts(xs[rank], topw, topi, w13, w2, 0, E)
    return {"err": float((out - ref).abs().max())}


def test_ep_alltoall_matches_single_rank():
    for r in run_ranks("ep_alltoall"):
        assert r["err"] < 1e-4


def collectives(rank, world):
    from mlopamd.parallel.comm import make_parallel_state

    ps = make_parallel_state(tp_size=2)
    x = torch.full((2, 3), float(rank + 1))
    ps.tp.all_reduce(x)
    g = ps.tp.all_gather(torch.tensor([[rank]]), dim=-1)
    b = torch.tensor([rank * 10.0])
    ps.tp.broadcast(b, 0)
    return {"ar": x.tolist(), "ag": g.tolist(), "b": b.item()}


def test_group_collectives():
    for r in run_ranks("collectives"):
        assert r["ar"] == [[3.0] * 3] * 2 and r["ag"] == [[0, 1]] and r["b"] == 0.0


def _ep_engine(rank, world):
    """DP attention + EP MoE (config 5): every rank schedules its OWN requests; the MoE
    layers exchange routed rows with sync-free fixed-capacity all-to-alls."""
    from mlopamd.models import build_model
    from mlopamd.models.config import get_config
    from mlopamd.parallel.comm import make_parallel_state
    from mlopamd.runtime.engine import Engine, EngineConfig
    from mlopamd.runtime.sampler import SamplingParams

    cfg = get_config("tiny-mixtral")
    full = build_model(cfg, device="cpu", dtype=torch.float32, seed=4)
    ps = make_parallel_state(tp_size=1, ep_size=world)
    assert ps.tp.size == 1 and ps.ep.size == world and ps.ep_cpu is not None
    shard = build_model(cfg, device="cpu", dtype=torch.float32, pstate=ps, seed=4).load_shard_from(full)
    assert shard.n_local_experts == cfg.num_experts // world
    ec = EngineConfig(max_num_seqs=4, max_num_batched_tokens=32, max_model_len=128, num_kv_blocks=40,
                      use_graphs=False)
    # uneven load: rank 0 gets three prompts (one long: chunked prefill), the last rank none
    mine = {0: PROMPTS, 1: [[7, 8, 9, 10, 11]]}.get(rank, []) if rank < world - 1 or world == 2 else []
    params = SamplingParams(max_tokens=6, ignore_eos=True)
    eng = Engine(shard, ec)
    outs = eng.generate(mine, params)
    ref = Engine(full, ec).generate(mine, params) if mine else []
    return {"ep": outs, "ref": ref, "idle_steps": eng.stats["ep_idle_steps"]}


def ep2_engine(rank, world):
    return _ep_engine(rank, world)


def ep4_engine(rank, world):
    return _ep_engine(rank, world)


@pytest.mark.parametrize("fn,world", [("ep2_engine", 2), ("ep4_engine", 4)])
def test_ep_engine_matches_single_rank(fn, world):
    res = run_ranks(fn, world)
    for r in res:
        assert r["ep"] == r["ref"]
    assert res[-1]["idle_steps"] > 0  # the idle rank joined every step's all-to-alls


def _overlap_rowpar(rank, world):
    """parallel/overlap.py: the chunked row-parallel projection (GEMM of chunk i+1 under the
    all-reduce + add + RMSNorm of chunk i on GPU) == the unchunked GEMM -> all-reduce -> norm,
    including a ragged last chunk, residual updated in place the same way (bit for bit at 2
    ranks; at 4 gloo's ring segments by message size, so the fp32 sum order may differ)."""
    from mlopamd import ops
    from mlopamd.parallel.comm import make_parallel_state
    from mlopamd.parallel.overlap import chunks_of, row_parallel_add_norm

    ps = make_parallel_state(tp_size=world)
    g = torch.Generator().manual_seed(rank)
    M, K, N = 700, 48, 64
    a = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=torch.Generator().manual_seed(100 + rank))
    res0 = torch.randn(M, N, generator=torch.Generator().manual_seed(7))  # same on every rank
    nw = torch.rand(N, generator=torch.Generator().manual_seed(8)) + 0.5
    r1, r2 = res0.clone(), res0.clone()
    assert len(chunks_of(M, 256)) == 3
    x1 = row_parallel_add_norm(a, w, ps.tp, r1, nw, 1e-5, chunk=256, min_rows=512)
    o = ops.gemm(a, w)
    ps.tp.all_reduce(o)
    x2 = ops.add_rmsnorm(o, r2, nw, 1e-5)
    return {"x": float((x1 - x2).abs().max()), "r": float((r1 - r2).abs().max())}


def overlap2(rank, world):
    return _overlap_rowpar(rank, world)


def overlap4(rank, world):
    return _overlap_rowpar(rank, world)


@pytest.mark.parametrize("fn,world", [("overlap2", 2), ("overlap4", 4)])
def test_chunked_row_parallel_matches_unchunked(fn, world):
    for r in run_ranks(fn, world):
        tol = 0.0 if world == 2 else 1e-4
        assert r["x"] <= tol and r["r"] <= tol, r


def _chan_stress(rank, world):
    """parallel/comm.HostChannel (ops/csrc/shm_channel.cc): one producer, world-1 consumers,
    far more messages than ring slots (back-pressure), every consumer sees every message in
    order; the segment name is already unlinked once every rank mapped it."""
    import glob

    from mlopamd.parallel.comm import HostChannel

    import torch.distributed as dist

    cpu = dist.new_group(list(range(world)), backend="gloo")
    ch = HostChannel(cpu, words=9)
    dist.barrier(group=cpu)  # rank 0 unlinked the name right after the construction barrier
    leftover = glob.glob("/dev/shm/mlop-chan-*")
    n, got = 5000, []
    v = torch.zeros(9, dtype=torch.int64)
    for i in range(n):
        if rank == 0:
            v[:] = torch.arange(9, dtype=torch.int64) + 9 * i
            ch.send(v)
        else:
            ch.recv(v)
            got.append(int(v[0]) == 9 * i and int(v[8]) == 9 * i + 8)
    ch.close()
    return {"ok": all(got) if rank else True, "n": len(got), "leftover": leftover}


def chan2(rank, world):
    return _chan_stress(rank, world)


def chan4(rank, world):
    return _chan_stress(rank, world)


@pytest.mark.parametrize("fn,world", [("chan2", 2), ("chan4", 4)])
def test_host_channel_broadcast(fn, world):
    res = run_ranks(fn, world)
    assert all(r["ok"] for r in res) and all(r["n"] == 5000 for r in res[1:])
    assert not any(r["leftover"] for r in res)


def _chan_fallback(rank, world, fail_rank):
    """a HostChannel that one rank cannot create / map raises ``Unavailable`` on
    EVERY rank (no rank left waiting in a broadcast or barrier), nothing is left in /dev/shm,
    and the TP engine's StepSync falls back to the gloo header: TP still == TP=1."""
    import glob

    import torch.distributed as dist

    from mlopamd.parallel.comm import HostChannel

    def broken(self, name):
        raise OSError("injected: no such shm namespace")

    if rank == fail_rank:
        HostChannel._open = broken
        HostChannel._create = broken
    cpu = dist.new_group(list(range(world)), backend="gloo")
    try:
        HostChannel(cpu, words=4)
        raised = False
    except HostChannel.Unavailable:
        raised = True
    dist.barrier(group=cpu)
    leftover = glob.glob("/dev/shm/mlop-chan-*")
    res = _tp_engine("tiny-llama")
    res.update(raised=raised, leftover=leftover)
    return res


def chan_fail_worker(rank, world):
    return _chan_fallback(rank, world, 1)


def chan_fail_leader(rank, world):
    return _chan_fallback(rank, world, 0)


@pytest.mark.parametrize("fn", ["chan_fail_worker", "chan_fail_leader"])
def test_host_channel_failure_falls_back_together(fn):
    r0, r1 = run_ranks(fn, 2)
    assert r0["raised"] and r1["raised"] and not r0["leftover"] and not r1["leftover"]
    assert r0["tp"] == r0["ref"] and r1["worker_steps"] > 0


def _xg_stress(rank, world):
    """parallel/comm.HostAllGather (ops/csrc/shm_allgather.cc): lock-step exchanges of
    variable-length messages (0 .. max_words words, the ring of 2 slots reused 2000 times), a
    rank that arrives late (the others' waits time out in their 250 ms slices and RESUME the same
    exchange), every rank sees every rank's words in order; nothing is left in /dev/shm; the
    gloo fallback gives the same answers."""
    import glob
    import time

    import torch.distributed as dist

    from mlopamd.parallel.comm import GlooAllGather, HostAllGather

    cpu = dist.new_group(list(range(world)), backend="gloo")
    xg = HostAllGather(cpu, max_words=64)
    dist.barrier(group=cpu)
    leftover = glob.glob("/dev/shm/mlop-xg-*")
    ok = True
    for it in range(2000):
        n = (it * 7 + rank * 13) % 65
        v = torch.arange(n, dtype=torch.int64) + 1000 * rank + it
        if it in (5, 1200) and rank == world - 1:
            time.sleep(0.6)  # the others' first slices expire mid-exchange
        got = xg.exchange(v)
        for q in range(world):
            m = (it * 7 + q * 13) % 65
            ok &= got[q].numel() == m and (m == 0 or (int(got[q][0]) == 1000 * q + it and
                                                      int(got[q][-1]) == 1000 * q + it + m - 1))
    xg.close()
    gl = GlooAllGather(cpu, 64)
    g2 = gl.exchange(torch.arange(rank + 1, dtype=torch.int64))
    ok &= [x.tolist() for x in g2] == [list(range(q + 1)) for q in range(world)]
    return {"ok": bool(ok), "leftover": leftover}


def xg2(rank, world):
    return _xg_stress(rank, world)


def xg4(rank, world):
    return _xg_stress(rank, world)


@pytest.mark.parametrize("fn,world", [("xg2", 2), ("xg4", 4)])
def test_host_allgather(fn, world):
    res = run_ranks(fn, world)
    assert all(r["ok"] for r in res) and not any(r["leftover"] for r in res)
