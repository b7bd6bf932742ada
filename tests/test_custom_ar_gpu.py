"""K15 one-shot all-reduce (ops/csrc/allreduce.hip) on ONE MI355X: two processes
share cuda:0 and map each other's buffers through HIP IPC, so the epoch-flag
handshake, the parity double-buffering, in-place use and hipGraph capture are
exercised exactly as across xGMI peers (the fabric path itself needs a
multi-GPU node).  Messages of 512 KiB and more take the two-shot kernel
(reduce-scatter + all-gather over peer memory); small ones are also forced
through it.  Oracle: fp32 sum in rank order of the known per-rank inputs,
rounded once to bf16 — the kernel must match it bit for bit on every rank.  The
broadcast kernel (the TP step-metadata path) must deliver the root's bytes exactly, and the
all-gather kernel every rank's piece in rank order."""
import os
import socket
import tempfile
import time

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

SIZES = [8, 4096, 3 * 4096, 64 * 1024, 8000, 4096, 200 * 1024, 300 * 1024, 1 << 20, 1000 * 1024 + 8]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs(it, n, world):
    return [torch.randn(n, generator=torch.Generator().manual_seed(1000 * it + p)).to(torch.bfloat16)
            for p in range(world)]


def _oracle(xs):
    acc = torch.zeros(xs[0].numel(), dtype=torch.float32)
    for x in xs:
        acc += x.float()
    return acc.to(torch.bfloat16)


def _worker(rank, world, port, out_dir, split):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from mlopamd.parallel.custom_ar import CustomAllReduce

    car = CustomAllReduce(rank, world, torch.device("cuda", 0), group=None, max_bytes=8 << 20, split_data=split)
    res = {"eager": [], "inplace": [], "graph": [], "two_shot": []}
    try:
        for it, n in enumerate(SIZES):
            xs = _inputs(it, n, world)
            x = xs[rank].cuda()
            if rank == 1 and it % 2:
                time.sleep(0.05)  # uneven arrival: rank 0 spins on the flags meanwhile
            out = torch.empty_like(x)
            car.all_reduce(x, out)
            torch.cuda.synchronize()
            res["eager"].append(torch.equal(out.cpu(), _oracle(xs)))
        # two-shot forced at small / odd sizes (fewer 16-B units than ranks x blocks), in place
        # and out of place, interleaved with one-shot calls (shared per-block epochs)
        for it, n in enumerate([8, 24, 4096, 8000, 12288, 64 * 1024 + 8]):
            xs = _inputs(200 + it, n, world)
            x = xs[rank].cuda()
            out = torch.empty_like(x)
            car.all_reduce(x, out, two_shot=True)
            y = xs[rank].cuda()
            car.all_reduce(y, two_shot=it % 2 == 0)
            torch.cuda.synchronize()
            res["two_shot"].append(torch.equal(out.cpu(), _oracle(xs)) and torch.equal(y.cpu(), _oracle(xs)))
        # broadcast (the TP step metadata path): int32 buffers from either root, uneven arrival
        # on both sides, interleaved with all-reduces on the same epochs
        res["bcast"] = []
        for it, (n, root) in enumerate([(4, 0), (64, 1), (4096 * 4, 0), (1 << 20, 1), (12, 0), (300 * 1024, 0)]):
            src = torch.randint(-2 ** 31, 2 ** 31 - 1, (n,), generator=torch.Generator().manual_seed(700 + it),
                                dtype=torch.int32)
            buf = src.cuda() if rank == root else torch.full((n,), -1, dtype=torch.int32, device="cuda")
            if it % 3 == 1 and rank == root:
                time.sleep(0.05)
            if it % 3 == 2 and rank != root:
                time.sleep(0.05)
            car.broadcast(buf, root)
            xs = _inputs(300 + it, 4096, world)
            y = xs[rank].cuda()
            car.all_reduce(y)
            torch.cuda.synchronize()
            res["bcast"].append(torch.equal(buf.cpu(), src) and torch.equal(y.cpu(), _oracle(xs)))
        # all-gather (TP logits / greedy pairs): fp32 and int32 pieces, uneven arrival,
        # interleaved with all-reduces on the same epochs
        res["gather"] = []
        for it, n in enumerate([2, 4, 4096, 3 * 1000 + 1, 64 * 1024]):
            pieces = [torch.randn(n, generator=torch.Generator().manual_seed(900 + 10 * it + p)) for p in range(world)]
            if it % 2:
                pieces = [(1e6 * x).to(torch.int32) for x in pieces]
            if rank == 1 and it % 2:
                time.sleep(0.05)
            got = car.all_gather(pieces[rank].cuda())
            xs = _inputs(400 + it, 4096, world)
            y = xs[rank].cuda()
            car.all_reduce(y)
            torch.cuda.synchronize()
            res["gather"].append(torch.equal(got.cpu(), torch.stack(pieces)) and torch.equal(y.cpu(), _oracle(xs)))
        # under contention: a side stream keeps a GEMM running on this rank (uneven, per-iteration
        # amounts) while all-reduce, broadcast and all-gather run their flag protocols
        res["contention"] = []
        side = torch.cuda.Stream()
        na = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
        nc = torch.empty_like(na)
        for it in range(12):
            with torch.cuda.stream(side):
                for _ in range(1 + (it + rank) % 3):
                    torch.matmul(na, na, out=nc)
            xs = _inputs(600 + it, 64 * 1024 + 8 * it, world)
            x = xs[rank].cuda()
            car.all_reduce(x)
            root = it % world
            src = torch.randint(-2 ** 31, 2 ** 31 - 1, (4096,), generator=torch.Generator().manual_seed(650 + it),
                                dtype=torch.int32)
            buf = src.cuda() if rank == root else torch.full((4096,), -1, dtype=torch.int32, device="cuda")
            car.broadcast(buf, root)
            pieces = [torch.randn(1000 + it, generator=torch.Generator().manual_seed(700 + 10 * it + p))
                      for p in range(world)]
            got = car.all_gather(pieces[rank].cuda())
            torch.cuda.synchronize()
            res["contention"].append(torch.equal(x.cpu(), _oracle(xs)) and torch.equal(buf.cpu(), src) and
                                     torch.equal(got.cpu(), torch.stack(pieces)))
        side.synchronize()
        # all-reduce + residual add (the TP decode norm chain): residual = bf16(residual +
        # bf16(sum)), interleaved with plain all-reduces on the same epochs, uneven arrival
        res["add"] = []
        for it, n in enumerate([8, 4096, 8192 * 4, 4 * 8192, 8000, 64 * 1024]):
            xs = _inputs(500 + it, n, world)
            r0 = torch.randn(n, generator=torch.Generator().manual_seed(550 + it)).to(torch.bfloat16)
            x, r = xs[rank].cuda(), r0.cuda()
            if rank == 1 and it % 2:
                time.sleep(0.05)
            car.all_reduce_add(x, r)
            ys = _inputs(560 + it, 4096, world)
            y = ys[rank].cuda()
            car.all_reduce(y)
            torch.cuda.synchronize()
            exp = (r0.float() + _oracle(xs).float()).to(torch.bfloat16)
            res["add"].append(torch.equal(r.cpu(), exp) and torch.equal(x.cpu(), xs[rank]) and
                              torch.equal(y.cpu(), _oracle(ys)))
        # in place, back to back (parity reuse every second call)
        for it in range(6):
            xs = _inputs(50 + it, 4096, world)
            x = xs[rank].cuda()
            car.all_reduce(x)
            torch.cuda.synchronize()
            res["inplace"].append(torch.equal(x.cpu(), _oracle(xs)))
        # hipGraph: capture two calls, replay with fresh inputs
        static = torch.zeros(2, 8192, dtype=torch.bfloat16, device="cuda")
        outs = torch.zeros_like(static)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        resid = torch.zeros(8192, dtype=torch.bfloat16, device="cuda")
        with torch.cuda.graph(g, stream=s):
            car.all_reduce(static[0], outs[0])
            car.all_reduce(static[1], outs[1], two_shot=True)
            car.all_reduce_add(static[0], resid)
        dist.barrier()
        for it in range(4):
            xs0, xs1 = _inputs(80 + it, 8192, world), _inputs(90 + it, 8192, world)
            r0 = torch.randn(8192, generator=torch.Generator().manual_seed(95 + it)).to(torch.bfloat16)
            static[0].copy_(xs0[rank].cuda())
            static[1].copy_(xs1[rank].cuda())
            resid.copy_(r0.cuda())
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            res["graph"].append(torch.equal(outs[0].cpu(), _oracle(xs0)) and
                                torch.equal(outs[1].cpu(), _oracle(xs1)) and
                                torch.equal(resid.cpu(), (r0.float() + _oracle(xs0).float()).to(torch.bfloat16)))
        res["error"] = car.error()
        res["uncached"] = car.uncached
        res["data_cached"] = car.data_cached
    finally:
        torch.cuda.synchronize()
        dist.barrier()
        car.close()
        dist.destroy_process_group()
    torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))


@pytest.mark.parametrize("world,split", [(2, True), (2, False), (8, True), (8, False)])
def test_custom_all_reduce_two_processes_one_gpu(world, split):
    """world = 8: the NR = 8 kernels (Llama-3-70B TP = 8) with 8 processes sharing the GPU.
    ``split``: the data parities in their own cached buffer (flags alone uncached) vs one
    uncached buffer for both -- every kernel bit-exact either way."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    d = tempfile.mkdtemp()
    mp.start_processes(_worker, args=(world, _free_port(), d, split), nprocs=world, join=True, start_method="spawn")
    for r in range(world):
        res = torch.load(os.path.join(d, f"r{r}.pt"), weights_only=False)
        assert res["error"] == 0, f"rank {r}: a flag wait timed out"
        # the flags a peer rewrites live in uncached memory (no stale L2 copy can be polled)
        assert res["uncached"], f"rank {r}: IPC flag buffer fell back to cached hipMalloc memory"
        assert res["data_cached"] == split
        assert all(res["eager"]), (r, res["eager"])
        assert all(res["inplace"]), (r, res["inplace"])
        assert all(res["graph"]), (r, res["graph"])
        assert all(res["two_shot"]), (r, res["two_shot"])
        assert all(res["bcast"]), (r, res["bcast"])
        assert all(res["gather"]), (r, res["gather"])
        assert all(res["contention"]), (r, res["contention"])
        assert all(res["add"]), (r, res["add"])


def _selfcheck_worker(rank, world, port, out_dir, inject):
    """make_parallel_state's first-contact check (custom_ar.py self_check / agree) on the gloo
    group: clean -> every rank keeps K15 ("ok"); one rank's K15 output perturbed
    (MLOP_INJECT_CAR_CORRUPT) -> EVERY rank falls back to the process-group path, and the
    fallback all-reduce still gives the right sum."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MLOP_CUSTOM_AR="force")
    if inject is not None:
        os.environ["MLOP_INJECT_CAR_CORRUPT"] = str(inject)
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from mlopamd.parallel.comm import make_parallel_state

    ps = make_parallel_state(tp_size=world)
    res = {"status": ps.tp.car_status, "has_car": ps.tp.car is not None, "check": ps.tp.car_check}
    xs = _inputs(7, 4096, world)
    x = xs[rank].cuda()
    if ps.tp.car is None:  # gloo fallback carries CPU tensors in this rehearsal
        xc = x.float().cpu()
        dist.all_reduce(xc)
        res["sum_ok"] = bool(torch.allclose(xc, sum(t.float() for t in xs), atol=1e-2))
    else:
        ps.tp.all_reduce(x)
        torch.cuda.synchronize()
        res["sum_ok"] = bool(torch.equal(x.cpu(), _oracle(xs)))
        ps.tp.car.close()
    dist.barrier()
    dist.destroy_process_group()
    torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))


@pytest.mark.parametrize("inject", [None, 1])
def test_custom_all_reduce_self_check_and_group_fallback(inject):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    d = tempfile.mkdtemp()
    world = 2
    mp.start_processes(_selfcheck_worker, args=(world, _free_port(), d, inject), nprocs=world, join=True,
                       start_method="spawn")
    rs = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=False) for r in range(world)]
    for r, res in enumerate(rs):
        assert res["sum_ok"], (r, res)
        if inject is None:
            assert res["status"] == "ok" and res["has_car"], (r, res)
            assert res["check"]["ok"] and all(res["check"]["checks"].values()), (r, res)
        else:
            # only rank 1's own one-shot check failed, yet the whole group fell back
            assert res["status"] == "fallback" and not res["has_car"], (r, res)
            assert res["check"]["checks"]["one_shot"] == (r != inject), (r, res)
