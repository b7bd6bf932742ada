"""K15 memory-layout microbench on ONE GPU: what the data path of the
custom all-reduce costs with its data parities in UNCACHED memory (one buffer: flags + data)
vs in their own CACHED buffer (flags alone uncached), at the two-shot kernel's prefill sizes
(1-64 MiB) and the one-shot kernel's decode sizes (16 KiB-4 MiB).

Two processes share cuda:0 and map each other's buffers over HIP IPC (as the GPU tests do), so
the publish stores, the peer reads and the flag protocol run exactly as across xGMI peers; only
the fabric hop itself is local HBM here.  Baseline: both processes doing a plain device copy
of the message at the same time (what the two-shot kernel's memory traffic would cost with no
protocol at all: it moves ~3x the message through HBM per rank).

Usage (GPU box): python scripts/bench_car.py [--iters 20]  -> a markdown table on stdout.
"""
from __future__ import annotations

import argparse
import os
import socket
import sys
import tempfile

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

TWO_SHOT_MIB = [1, 2, 4, 8, 16, 32, 64]
ONE_SHOT_KIB = [16, 64, 256, 1024, 4096]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _time(fn, iters, barrier):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    barrier()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    barrier()
    return a.elapsed_time(b) * 1e3 / iters  # us per call


def _worker(rank, world, port, out_dir, iters):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from mlopamd.parallel.custom_ar import CustomAllReduce

    res = {}
    bar = dist.barrier
    try:
        for split in (False, True):
            car = CustomAllReduce(rank, world, torch.device("cuda", 0), max_bytes=128 << 20, split_data=split)
            for mib in TWO_SHOT_MIB:
                n = (mib << 20) // 2
                x = torch.randn(n, device="cuda").to(torch.bfloat16)
                out = torch.empty_like(x)
                res[("two", split, mib)] = _time(lambda: car.all_reduce(x, out, two_shot=True), iters, bar)
            for kib in ONE_SHOT_KIB:
                n = (kib << 10) // 2
                x = torch.randn(n, device="cuda").to(torch.bfloat16)
                out = torch.empty_like(x)
                res[("one", split, kib)] = _time(lambda: car.all_reduce(x, out, two_shot=False), iters, bar)
            res[("err", split)] = car.error()
            torch.cuda.synchronize()
            bar()
            car.close()
        for mib in TWO_SHOT_MIB:
            n = (mib << 20) // 2
            x = torch.randn(n, device="cuda").to(torch.bfloat16)
            y = torch.empty_like(x)
            res[("copy", mib)] = _time(lambda: y.copy_(x), iters, bar)
    finally:
        dist.destroy_process_group()
    torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    d = tempfile.mkdtemp()
    mp.start_processes(_worker, args=(2, _free_port(), d, a.iters), nprocs=2, join=True, start_method="spawn")
    rs = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(2)]

    def t(key):  # the slower rank's time per call
        return max(r[key] for r in rs)

    assert all(r[("err", s)] == 0 for r in rs for s in (False, True)), "a flag wait timed out"
    print("## two-shot all-reduce, 2 ranks on one GPU (us per call; GB/s = message bytes / time)\n")
    print("| message | uncached data | cached data (split) | split / uncached | both ranks' plain copy |")
    print("|---|---|---|---|---|")
    for mib in TWO_SHOT_MIB:
        u, c, cp = t(("two", False, mib)), t(("two", True, mib)), t(("copy", mib))
        gb = (mib << 20) / 1e3
        print(f"| {mib} MiB | {u:.1f} ({gb / u:.0f} GB/s) | {c:.1f} ({gb / c:.0f} GB/s) | {c / u:.2f} | "
              f"{cp:.1f} |")
    print("\n## one-shot all-reduce (decode sizes)\n")
    print("| message | uncached data | cached data (split) | split / uncached |")
    print("|---|---|---|---|")
    for kib in ONE_SHOT_KIB:
        u, c = t(("one", False, kib)), t(("one", True, kib))
        print(f"| {kib} KiB | {u:.1f} | {c:.1f} | {c / u:.2f} |")


if __name__ == "__main__":
    main()
