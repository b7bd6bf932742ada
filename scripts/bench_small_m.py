"""Small-M (batch 5-64 decode) projection GEMMs: every small tiling the planner can launch, forced
through ``gemm_dense_plan`` (tile, K splits, LDS ring depth), on the Llama-3-8B projections.
These GEMMs stream the weights, so each line also gives the weight bytes per second of the best
candidate and of the planner's own choice ("auto"), with the weights cold (a rotation over > 1 GB
of copies, as in serving where 16 GB of other layers pass between two calls of one matrix).
One process, interleaved rounds, random data.

Usage (GPU box): python scripts/bench_small_m.py [--ms 8,16,32,64] [--shapes qkv,o,gate_up,down]
       --nt: the planner's tile only, default vs non-temporal weight loads (gemm_small_nt), 4 rounds
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlopamd import ops  # noqa: E402

PROJ = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


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


def candidates(M):
    bm = 16 if M <= 16 else 32 if M <= 32 else 64
    out = [("auto", -1, -1, -1, -1, 0)]
    for bn, st, sp in itertools.product((32, 64), (4, 6, 8), (1, 2, 3, 4, 6, 8)):
        if bm == 64 and bn == 32 and st != 4:
            continue  # 64x32 has one ring depth
        if bm == 32 and bn == 32 and st == 6:
            continue
        out.append((f"{bm}x{bn}/s{st}/k{sp}", 0, bm, bn, sp, st))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="8,16,32,64")
    ap.add_argument("--shapes", default="qkv,o,gate_up,down")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--nt", action="store_true")
    a = ap.parse_args()
    ops.load()
    dev = torch.device("cuda")
    ops._sk_reserve(dev)
    for M in [int(m) for m in a.ms.split(",")]:
        for name in a.shapes.split(","):
            N, K = PROJ[name]
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            # serving streams every layer's weights from HBM: cycle through copies totalling
            # > 1 GB so no call finds its weights in the 256 MB MALL (a loop over one matrix of
            # 33-235 MB measures the cache, not HBM)
            ncp = max(2, (1 << 30) // (N * K * 2) + 1)
            ws = [(0.02 * torch.randn(N, K, device=dev)).to(torch.bfloat16) for _ in range(ncp)]
            w = ws[0]
            epi = ops.EPI_SILU_MUL if name == "gate_up" else ops.EPI_NONE
            cyc = [0]

            def run():
                cyc[0] = (cyc[0] + 1) % ncp
                return ops.gemm(x, ws[cyc[0]], epi=epi)

            res, ref = {}, None
            cands = candidates(M)
            if a.nt:
                cands = [("auto", -1, -1, -1, -1, 0, 0), ("auto_nt", -1, -1, -1, -1, 0, 1)]
            else:
                cands = [c + (torch.ops.mlop.gemm_small_nt(-1),) for c in cands]
            for _ in range(4 if a.nt else 2):
                for label, v, bm, bn, sp, st, nt in cands:
                    prev_nt = torch.ops.mlop.gemm_small_nt(-1)
                    try:
                        torch.ops.mlop.gemm_small_nt(nt)
                        torch.ops.mlop.gemm_dense_plan(v, bm, bn, sp, st)
                        ops.GEMM_BACKEND = "mlop"
                        y = ops.gemm(x, w, epi=epi)
                        if ref is None:
                            ref = y.float()
                        ok = float((y.float() - ref).abs().max()) <= 0.05 * float(ref.abs().max()) + 1e-3
                        t = timeit(run, a.iters)
                        res[label] = min(res.get(label, 1e9), t) if ok else -1.0
                    finally:
                        ops.GEMM_BACKEND = ops.GEMM_BACKEND_DEFAULT
                        torch.ops.mlop.gemm_dense_plan(-1, -1, -1, -1, 0)
                        torch.ops.mlop.gemm_small_nt(prev_nt)
            good = {k: v for k, v in res.items() if v > 0}
            best = min(good, key=good.get)
            wbytes = N * K * 2
            top = sorted(good.items(), key=lambda kv: kv[1])[:5]
            print(json.dumps(dict(shape=name, M=M, auto_us=round(res["auto"], 1), best=best,
                                  best_us=round(good[best], 1), best_tbs=round(wbytes / good[best] / 1e6, 2),
                                  auto_tbs=round(wbytes / res["auto"] / 1e6, 2),
                                  top5={k: round(v, 1) for k, v in top},
                                  bad=[k for k, v in res.items() if v < 0])), flush=True)
            del x, w, ws


if __name__ == "__main__":
    main()
