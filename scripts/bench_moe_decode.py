"""Mixtral-8x7B MoE grouped GEMMs at DECODE routing shapes: per plan
candidate, the grouped gate_up (SiLU epilogue, N = 28672, K = 4096) and down (N = 4096,
K = 14336) time, the expert-weight stream rate (bytes of every expert with routed rows / time)
and TFLOP/s, on the routing the engine sees:

  * ROWS = 2 x decode tokens (top-2), split over 8 experts multinomially (seeded): 128 rows =
    batch 64, 2048 rows = the decode-only steps of batch 1024 (~256 +- 16 rows per expert).

Candidates are forced through ``gemm_grouped_plan`` (BM, BN, ring stages, K splits; -1 = the
planner's own choice) so one process compares them interleaved on one GPU.

Usage (GPU box): python scripts/bench_moe_decode.py [--rows 128,2048] [--iters 10]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlopamd import ops  # noqa: E402

E = 8
# (label, BM, BN, stages, splits); -1 = planner default
CANDIDATES = {
    "small": [("auto", -1, -1, -1, -1), ("16x64/s6", 16, 64, 6, -1), ("16x64/s8", 16, 64, 8, -1),
              ("32x64/s6", 32, 64, 6, -1), ("32x32/s8", 32, 32, 8, -1), ("64x64/s6", 64, 64, 6, -1),
              ("64x64/s4", 64, 64, 4, -1), ("64x64/s3", 64, 64, 3, -1), ("64x32/s4", 64, 32, 4, -1),
              ("32x64/s6/k1", 32, 64, 6, 1), ("32x64/s6/k4", 32, 64, 6, 4), ("64x64/s3/k1", 64, 64, 3, 1),
              ("64x64/s3/k2", 64, 64, 3, 2), ("64x64/s3/k4", 64, 64, 3, 4), ("64x64/s6/k4", 64, 64, 6, 4),
              ("16x64/s8/k2", 16, 64, 8, 2), ("16x64/s8/k4", 16, 64, 8, 4)],
    "mid": [("auto", -1, -1, -1, -1), ("128x64", 128, 64, -1, -1), ("64x64/s6", 64, 64, 6, -1),
            ("64x64/s3", 64, 64, 3, -1), ("256x128", 256, 128, -1, 1), ("256x64", 256, 64, -1, 1),
            ("256x256", 256, 256, -1, 1)],
    "large": [("auto", -1, -1, -1, -1), ("auto+bal", -1, -1, -1, -1), ("auto+bal2", -1, -1, -1, -1), ("256x128", 256, 128, -1, 1),
              ("256x64", 256, 64, -1, 1), ("128x64", 128, 64, -1, 1), ("256x256", 256, 256, -1, 1)],
}


def timeit(fn, iters):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="128,256,512,2048")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--counts", default="",
                    help="explicit per-expert row counts instead of --rows, ';'-separated sets of 8 "
                         "comma-separated counts (e.g. '256,256,256,256,256,256,256,256;257,...')")
    a = ap.parse_args()
    ops.load()
    dev = torch.device("cuda")
    bf = torch.bfloat16
    ops._sk_reserve(dev)
    bal_default = torch.ops.mlop.gemm_grouped_balance(-1)
    rng = np.random.default_rng(0)
    shapes = (("gate_up", 28672, 4096, 1), ("down", 4096, 14336, 0))
    ws = {name: (0.02 * torch.randn(E, N, K, device=dev)).to(bf) for name, N, K, _ in shapes}
    sets = ([np.array([int(c) for c in cs.split(",")]) for cs in a.counts.split(";")] if a.counts else
            [rng.multinomial(int(r), [1 / E] * E) for r in a.rows.split(",")])
    for counts in sets:
        rows = int(counts.sum())
        off = torch.tensor([0] + list(np.cumsum(counts)), device=dev, dtype=torch.int32)
        group = "small" if rows // E <= 32 else ("mid" if rows // E <= 128 else "large")
        for name, N, K, epi in shapes:
            x = torch.randn(rows, K, device=dev, dtype=bf)
            w = ws[name]
            ref = None
            best = {}
            for _ in range(2):  # interleaved rounds
                for label, bm, bn, st, sp in CANDIDATES[group]:
                    torch.ops.mlop.gemm_grouped_plan(bm, bn, st, sp)
                    # "+bal" / "+bal2": equal row ranges per expert m-tile, + the 16-row MFMA skip
                    # (gemm_grouped_balance 1 / 2); every other candidate runs with 0
                    torch.ops.mlop.gemm_grouped_balance(2 if label.endswith("+bal2") else 1 if label.endswith("+bal") else 0)
                    try:
                        y = ops.grouped_gemm(x, w, off, epi=epi, avg_rows=rows // E)
                        if ref is None:
                            ref = y.float()
                        err = float((y.float() - ref).abs().max())
                        t = timeit(lambda: ops.grouped_gemm(x, w, off, epi=epi, avg_rows=rows // E), a.iters)
                    except RuntimeError as e:  # a candidate the launcher has no config for
                        best[label] = (None, str(e)[:80])
                        continue
                    if label not in best or (best[label][0] is not None and t < best[label][0]):
                        best[label] = (t, err)
            torch.ops.mlop.gemm_grouped_plan(-1, -1, -1, -1)
            torch.ops.mlop.gemm_grouped_balance(bal_default)
            wbytes = int((counts > 0).sum()) * N * K * 2
            for label, (t, err) in best.items():
                if t is None:
                    print(json.dumps(dict(shape=name, rows=rows, plan=label, error=err)), flush=True)
                    continue
                print(json.dumps(dict(shape=name, rows=rows, counts=counts.tolist(), plan=label, us=round(t, 1),
                                      weight_tbs=round(wbytes / t / 1e6, 2),
                                      tflops=round(2 * rows * N * K / t / 1e6, 1), max_abs_diff=err)), flush=True)
            del x


if __name__ == "__main__":
    main()
