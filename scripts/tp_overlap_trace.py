#!/usr/bin/env python3
"""TP=2 on ONE GPU (two processes, gloo + the K15 IPC all-reduce): the chunked row-parallel
projection of parallel/overlap.py at a Llama-3-70B TP-shard shape, for a rocprofv3 kernel trace
that shows chunk i+1's GEMM running while chunk i's all-reduce (car_twoshot_kernel) and
add + RMSNorm run on the communication stream.  Also times chunked vs unchunked per rank.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_tp -o tp -- python3 scripts/tp_overlap_trace.py
    python3 scripts/tp_overlap_trace.py --analyze gpurun_out/prof_tp   # overlap summary of the traces
"""
import argparse
import csv
import glob
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _worker(rank, world, port, M, K, N, iters):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MLOP_CUSTOM_AR="force")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from mlopamd import ops
    from mlopamd.parallel.comm import make_parallel_state
    from mlopamd.parallel.overlap import row_parallel_add_norm

    ps = make_parallel_state(tp_size=world)
    dev = torch.device("cuda", 0)
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (0.02 * torch.randn(N, K, device=dev)).to(torch.bfloat16)
    res = torch.randn(M, N, device=dev).to(torch.bfloat16)
    nw = torch.ones(N, device=dev, dtype=torch.bfloat16)
    times = {}
    for mode in ("chunked", "unchunked", "chunked"):
        for _ in range(2):  # warm-up
            row_parallel_add_norm(a, w, ps.tp, res, nw, 1e-5, min_rows=1 if mode == "chunked" else 1 << 30)
        torch.cuda.synchronize()
        dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            row_parallel_add_norm(a, w, ps.tp, res, nw, 1e-5, min_rows=1 if mode == "chunked" else 1 << 30)
        e1.record()
        torch.cuda.synchronize()
        times[mode] = round(e0.elapsed_time(e1) / iters * 1e3, 1)
    dist.barrier()
    if rank == 0:
        print(f"[tp_overlap] M={M} K={K} N={N} world={world}: us per call {times} "
              f"(the two ranks share one GPU: absolute times include the other rank's work)", flush=True)
    ps.tp.car.close()
    dist.destroy_process_group()


def analyze(d):
    """Per process trace: time during which a GEMM kernel and an all-reduce kernel overlap."""
    for f in sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)):
        by_pid = {}
        with open(f) as fh:
            for r in csv.DictReader(fh):
                by_pid.setdefault(r.get("Process_Id", "0"), []).append(
                    (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
        for pid, rs in by_pid.items():
            gemm = [(s, e) for s, e, n in rs if "gemm" in n]
            ar = [(s, e) for s, e, n in rs if "car_" in n]
            ov = 0
            for s1, e1 in ar:
                for s2, e2 in gemm:
                    ov += max(0, min(e1, e2) - max(s1, s2))
            ar_t = sum(e - s for s, e in ar)
            print(f"{os.path.basename(f)} pid {pid}: {len(gemm)} GEMM / {len(ar)} all-reduce kernels; "
                  f"all-reduce time {ar_t / 1e6:.2f} ms, of it under a GEMM {ov / 1e6:.2f} ms "
                  f"({100 * ov / max(ar_t, 1):.0f} %)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--analyze", default=None)
    ap.add_argument("--M", type=int, default=2048)  # unchunked 32 MiB: still on the two-shot kernel
    ap.add_argument("--K", type=int, default=1024)   # 70B TP=8 O projection: K = 8192 / 8
    ap.add_argument("--N", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    if a.analyze:
        return analyze(a.analyze)
    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_worker, args=(2, port, a.M, a.K, a.N, a.iters), nprocs=2, join=True, start_method="spawn")


if __name__ == "__main__":
    main()
