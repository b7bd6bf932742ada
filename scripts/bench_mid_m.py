"""Mid-M projection GEMMs: every hand-written tiling the planner can pick,
forced one at a time through ``gemm_dense_plan``, against hipBLASLt (torch.matmul) on the
Llama-3-8B projections at the row counts of batch 512-1024 serving (decode rows + prompt
chunks of the mixed steps).  One process, interleaved rounds, random data.

Prints one JSON line per (shape, M): every candidate's us, the planner's own choice ("auto")
and the library's, so a per-shape table (and what the planner should pick) falls out.

Usage (GPU box): python scripts/bench_mid_m.py [--ms 512,1024,...] [--shapes qkv,o,...] [--cold]
  --cold: rotate over > 1 GB of weight copies (decode-sized M streams its weights from HBM in
  serving; a loop over one matrix measures the MALL), plus split-K variants of the narrow tiles
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlopamd import ops  # noqa: E402

PROJ = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
        "lm_head": (128256, 4096)}
# (label, variant, BM, BN, splits): -1 = planner default
CANDS = [("auto", -1, -1, -1, -1), ("w4", 5, 256, 256, -1), ("w4h", 6, 128, 256, -1), ("pp", 3, 256, 256, -1),
         ("256x128", 0, 256, 128, 1), ("256x128/k2", 0, 256, 128, 2), ("256x64", 0, 256, 64, 1),
         ("128x64", 0, 128, 64, 1), ("256x256/2s", 1, 256, 256, 1)]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="512,768,1024,1536,2048,2304,2560,2816,3072,4608,6144,8704")
    ap.add_argument("--shapes", default="qkv,o,gate_up,down")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--cold", action="store_true")
    a = ap.parse_args()
    cands = list(CANDS)
    if a.cold:
        cands += [("256x128/k4", 0, 256, 128, 4), ("256x64/k2", 0, 256, 64, 2), ("256x64/k4", 0, 256, 64, 4),
                  ("128x64/k2", 0, 128, 64, 2), ("128x64/k4", 0, 128, 64, 4)]
    ops.load()
    dev = torch.device("cuda")
    ops._sk_reserve(dev)
    for M in [int(m) for m in a.ms.split(",")]:
        for name in a.shapes.split(","):
            N, K = PROJ[name]
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            ncp = max(2, (1 << 30) // (N * K * 2) + 1) if a.cold else 1
            ws = [(0.02 * torch.randn(N, K, device=dev)).to(torch.bfloat16) for _ in range(ncp)]
            w = ws[0]
            cyc = [0]

            def wnext():
                cyc[0] = (cyc[0] + 1) % ncp
                return ws[cyc[0]]
            epi = ops.EPI_SILU_MUL if name == "gate_up" else ops.EPI_NONE
            res, ref = {}, None
            for _ in range(2):
                for label, v, bm, bn, sp in cands:
                    try:
                        torch.ops.mlop.gemm_dense_plan(v, bm, bn, sp)
                        ops.GEMM_BACKEND = "mlop"
                        y = ops.gemm(x, w, epi=epi)
                        if ref is None:
                            ref = y.float()
                        ok = float((y.float() - ref).abs().max()) <= 0.05 * float(ref.abs().max()) + 1e-3
                        t = timeit(lambda: ops.gemm(x, wnext(), epi=epi), a.iters)
                        res[label] = min(res.get(label, 1e9), t) if ok else -1.0
                    finally:
                        ops.GEMM_BACKEND = ops.GEMM_BACKEND_DEFAULT
                        torch.ops.mlop.gemm_dense_plan(-1, -1, -1, -1)
                if epi == ops.EPI_NONE:
                    t = timeit(lambda: torch.matmul(x, wnext().t()), a.iters)
                    res["hipblaslt"] = min(res.get("hipblaslt", 1e9), t)
            good = {k: v for k, v in res.items() if v > 0 and k != "hipblaslt"}
            best = min(good, key=good.get)
            line = dict(shape=name, M=M, N=N, K=K, us={k: round(v, 1) for k, v in res.items()}, best=best,
                        best_tflops=round(2 * M * N * K / good[best] / 1e6, 1))
            if "hipblaslt" in res:
                line["best_vs_lib"] = round(res["hipblaslt"] / good[best], 3)
                line["auto_vs_lib"] = round(res["hipblaslt"] / res["auto"], 3)
            print(json.dumps(line), flush=True)
            del x, w


if __name__ == "__main__":
    main()
