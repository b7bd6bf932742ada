"""Grouped MoE GEMM against dense GEMMs of the same work (Mixtral-8x7B gate_up / down at the
mixed-step sizes of batch 1024): how much of the grouped kernel's gap to the dense rate is
the grouping itself.  Per shape and ROWS_PER_EXPERT (env, comma list):

  * grouped / grouped_o1: 8 experts x R rows (`ops.grouped_gemm`, the ping-pong grouped kernel)
    in the slot-fastest / expert-major tile order (gemm_grouped_order 0 / 1);
  * dense_pp / dense_w4: ONE [8R, K] x [N, K] GEMM on the ping-pong kernel
    (gemm_big_variant 3) / the four-wave kernel (5, the default) -- the same FLOPs, one weight;
  * expert_pp: one expert's [R, K] x [N, K] on the ping-pong kernel, x 8 (serial launches).

Usage (GPU box): ROWS_PER_EXPERT=765,512 python scripts/bench_grouped_dense.py"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlopamd import ops  # noqa: E402

ops.load()
dev = torch.device("cuda")
bf = torch.bfloat16
E = 8
ops._sk_reserve(dev)


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def dense(x, w, epi, variant):
    prev = torch.ops.mlop.gemm_big_variant(variant)
    ops.GEMM_BACKEND = "mlop"
    try:
        return ops.gemm(x, w, epi=epi)
    finally:
        torch.ops.mlop.gemm_big_variant(prev)
        ops.GEMM_BACKEND = ops.GEMM_BACKEND_DEFAULT


def grouped(x, w, off, epi, R, order):
    prev = torch.ops.mlop.gemm_grouped_order(order)
    try:
        return ops.grouped_gemm(x, w, off, epi=epi, avg_rows=R)
    finally:
        torch.ops.mlop.gemm_grouped_order(prev)


for R in [int(r) for r in os.environ.get("ROWS_PER_EXPERT", "765").split(",")]:
    for name, N, K, epi in (("gate_up", 28672, 4096, ops.EPI_SILU_MUL), ("down", 4096, 14336, ops.EPI_NONE)):
        M = E * R
        x = torch.randn(M, K, device=dev, dtype=bf)
        w = (0.02 * torch.randn(E, N, K, device=dev)).to(bf)
        off = torch.tensor(np.arange(E + 1) * R, device=dev, dtype=torch.int32)
        flops = 2 * M * N * K
        res = {}
        for _ in range(2):  # interleaved rounds, best of
            cands = {
                "grouped": lambda: grouped(x, w, off, epi, R, 0),
                "grouped_o1": lambda: grouped(x, w, off, epi, R, 1),
                "dense_pp": lambda: dense(x, w[0], epi, 3),
                "dense_w4": lambda: dense(x, w[0], epi, 5),
                "expert_pp": lambda: [dense(x[e * R:(e + 1) * R], w[e], epi, 3) for e in range(E)],
            }
            for k, fn in cands.items():
                t = timeit(fn)
                res[k] = min(res.get(k, t), t)
        print(json.dumps(dict(shape=name, rows_per_expert=R, **{k: round(v, 1) for k, v in res.items()},
                              **{f"{k}_pf": round(flops / v / 1e9, 3) for k, v in res.items()})), flush=True)
        del x, w
