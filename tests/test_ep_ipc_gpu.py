"""Expert-parallel exchange over IPC peer memory (ops/csrc/ep_exchange.hip, parallel/ep_ipc.py)
on ONE MI355X: two processes share cuda:0 and map each other's buffers through HIP IPC, so the
count exchange, the exact expert-grouped placement, the three flag phases and hipGraph capture
run exactly as across xGMI peers (the fabric itself needs a multi-GPU node).

1. The exchange alone, bit-exact: every rank routes a different number of tokens; the rows a
   rank receives must be, expert by expert, the routed rows of rank 0 then rank 1 in slot order
   (the fp32 oracle rebuilds them from both ranks' inputs); a per-expert power-of-two scale
   stands in for the experts, so the combined output sum_j w_j * 2^e_j * x[t] has one rounding
   and must match the oracle bit for bit -- eagerly, with uneven arrival, and replayed from a
   captured hipGraph with fresh inputs.
2. The tiny-Mixtral engine at EP = 2 (DP attention: each rank serves its own prompts, one rank
   also idles) on the HIP path with decode graphs == the same engine eager, and its greedy tokens
   are the unsharded model's dense fp32 argmax (up to bf16 near-ties)."""
import os
import socket
import tempfile
import time

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

E, K, H, TCAP = 8, 2, 512, 64
TS = [37, 5]  # tokens per rank


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs(it, rank):
    g = torch.Generator().manual_seed(100 * it + rank)
    T = TS[rank] if it % 2 == 0 else TS[1 - rank]
    x = torch.randn(T, H, generator=g).to(torch.bfloat16)
    topi = torch.stack([torch.randperm(E, generator=g)[:K] for _ in range(T)]).to(torch.int32)
    topw = torch.rand(T, K, generator=g)
    return x, topi, topw / topw.sum(-1, keepdim=True)


def _experts(xp, offsets, n_local):
    """stand-in experts: local expert j scales its rows by 2^(j+1) (exact in bf16)"""
    y = torch.empty_like(xp)
    off = offsets.tolist()
    for j in range(n_local):
        y[off[j]:off[j + 1]] = xp[off[j]:off[j + 1]] * float(2 ** (j + 1))
    return y


def _oracle_received(rank, world, it, n_local):
    rows = []
    for x0 in range(rank * n_local, (rank + 1) * n_local):
        for s in range(world):
            x, topi, _ = _inputs(it, s)
            for slot in range(topi.numel()):
                if int(topi.view(-1)[slot]) == x0:
                    rows.append(x[slot // K])
    return torch.stack(rows) if rows else torch.zeros(0, H, dtype=torch.bfloat16)


def _oracle_out(it, rank, n_local):
    """(fused multiply-add, multiply-then-add) fp32 accumulations of sum_j w_j * y_j, j in
    order, each rounded once to bf16: the kernel's fp32 accumulate may or may not contract."""
    x, topi, topw = _inputs(it, rank)
    y = (2.0 ** ((topi % n_local) + 1)).double()[:, :, None] * x.double()[:, None, :]  # exact
    w = topw.double()[:, :, None]
    fma = torch.zeros(x.shape, dtype=torch.float32)
    mul = torch.zeros(x.shape, dtype=torch.float32)
    for j in range(K):
        fma = (fma.double() + w[:, j] * y[:, j]).float()
        mul = mul + (w[:, j] * y[:, j]).float()
    return fma.to(torch.bfloat16), mul.to(torch.bfloat16)


def _matches(out, oracle):
    a, b = oracle
    return bool(((out == a) | (out == b)).all())


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from mlopamd.parallel.ep_ipc import EPExchange

    ex = EPExchange(rank, world, E, K, H, TCAP, torch.device("cuda", 0))
    nl = E // world
    res = {"recv": [], "out": [], "graph": []}
    try:
        for it in range(6):
            x, topi, topw = _inputs(it, rank)
            if rank == 1 and it % 2:
                time.sleep(0.05)  # uneven arrival: rank 0 spins on the flags meanwhile
            xp, off = ex.dispatch(x.cuda(), topi.cuda(), max(TS))
            torch.cuda.synchronize()
            n = int(off[-1])
            res["recv"].append(torch.equal(xp[:n].cpu(), _oracle_received(rank, world, it, nl)))
            y = _experts(xp, off, nl)
            out = ex.combine(y, topw.cuda(), topi.cuda(), x.shape[0])
            torch.cuda.synchronize()
            res["out"].append(_matches(out.cpu(), _oracle_out(it, rank, nl)))
        # hipGraph: dispatch -> stand-in experts (device offsets, no host read) -> combine
        T = TS[rank]
        sx = torch.zeros(T, H, dtype=torch.bfloat16, device="cuda")
        si = torch.zeros(T, K, dtype=torch.int32, device="cuda")
        sw = torch.zeros(T, K, device="cuda")
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            xp, off = ex.dispatch(sx, si, max(TS))
            rows = torch.arange(xp.shape[0], device="cuda", dtype=torch.int32)
            j = torch.searchsorted(off[1:].contiguous(), rows, right=True)  # local expert of each row
            y = (xp.float() * torch.pow(2.0, (j + 1).float())[:, None]).to(torch.bfloat16)
            gout = ex.combine(y, sw, si, T)
        dist.barrier()
        for it in range(6, 10):
            x, topi, topw = _inputs(it, rank)
            if x.shape[0] != T:
                continue  # the graph's static T: every other iteration swaps the ranks' sizes
            sx.copy_(x.cuda())
            si.copy_(topi.cuda())
            sw.copy_(topw.cuda())
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            res["graph"].append(_matches(gout.cpu(), _oracle_out(it, rank, nl)))
        res["error"] = ex.error()
        res["uncached"] = ex.uncached
    finally:
        torch.cuda.synchronize()
        dist.barrier()
        ex.close()
        dist.destroy_process_group()
    torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))


def test_ep_exchange_two_processes_one_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    d = tempfile.mkdtemp()
    mp.start_processes(_worker, args=(2, _free_port(), d), nprocs=2, join=True, start_method="spawn")
    for r in range(2):
        res = torch.load(os.path.join(d, f"r{r}.pt"), weights_only=False)
        assert res["error"] == 0, f"rank {r}: a flag wait timed out or a capacity overflowed"
        assert res["uncached"], f"rank {r}: IPC buffer fell back to cached hipMalloc memory"
        assert all(res["recv"]), (r, res["recv"])
        assert all(res["out"]), (r, res["out"])
        assert res["graph"] and all(res["graph"]), (r, res["graph"])


PROMPTS = {0: [[5, 9, 11, 40, 2, 7], list(range(20, 61)), [100, 3]], 1: [list(range(300, 390))]}


def _engine_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from mlopamd.models import build_model
    from mlopamd.models.config import get_config
    from mlopamd.parallel.comm import make_parallel_state
    from mlopamd.runtime.engine import Engine, EngineConfig
    from mlopamd.runtime.sampler import SamplingParams

    dev = torch.device("cuda", 0)
    cfg = get_config("tiny-mixtral")
    full = build_model(cfg, device=dev, seed=4)
    ps = make_parallel_state(tp_size=1, ep_size=world)
    shard = build_model(cfg, device=dev, pstate=ps, seed=4).load_shard_from(full)
    res = {}
    try:
        for key, graphs in (("eager", False), ("graph", True)):
            ec = EngineConfig(max_num_seqs=4, max_num_batched_tokens=48, max_model_len=256, num_kv_blocks=64,
                              use_graphs=graphs, graph_buckets=(1, 2, 4))
            eng = Engine(shard, ec)
            assert ps.ep.ex is not None  # the IPC exchange, not RCCL / gloo all_to_all
            res[key] = eng.generate(PROMPTS[rank], SamplingParams(max_tokens=8, ignore_eos=True))
            res[key + "_graph_steps"] = eng.stats["graph_steps"]
            res[key + "_idle"] = eng.stats["ep_idle_steps"]
        res["error"] = ps.ep.ex.error()
    finally:
        torch.cuda.synchronize()
        dist.barrier()
        if ps.ep.ex is not None:
            ps.ep.ex.close()
        dist.destroy_process_group()
    torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))


def test_ep2_mixtral_engine_on_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    d = tempfile.mkdtemp()
    mp.start_processes(_engine_worker, args=(2, _free_port(), d), nprocs=2, join=True, start_method="spawn")
    from mlopamd.models import build_model
    from mlopamd.models.config import get_config
    from test_model_gpu import _check_greedy

    full = build_model(get_config("tiny-mixtral"), device=torch.device("cuda", 0), seed=4)
    for r in range(2):
        res = torch.load(os.path.join(d, f"r{r}.pt"), weights_only=False)
        assert res["error"] == 0
        assert res["graph_graph_steps"] > 0 and res["eager_graph_steps"] == 0
        assert res["graph"] == res["eager"], r  # decode-graph replay (exchange inside) == eager
        _check_greedy(full, PROMPTS[r], res["eager"])
