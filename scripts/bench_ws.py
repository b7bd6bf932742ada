"""Weight-streaming MFMA GEMM (ops/csrc/gemm_ws.hip) vs the planner's small-M tiles at decode
batch sizes, Llama-3-8B projections, cold weights (a rotation over > 1 GB of copies, as in
serving where 16 GB of other layers stream between two calls of one matrix), one process,
interleaved rounds.  Also checks each ws result against the fp32 torch product.

  plain forms:  qkv / o / down plain, gate_up with the SiLU-mul epilogue (ops.gemm vs gemm_ws)
  --chain:      the decode norm chain's forms too: gate_up / qkv-plain with the row-scale
                prologue (rs), o / down adding into a residual (epi 5)

Usage (GPU box): python scripts/bench_ws.py [--ms 8,16,32,64] [--shapes qkv,o,gate_up,down]
"""
from __future__ import annotations

import argparse
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


def ref_silu_mul(y):
    from mlopamd.ops import deinterleave_cols, reference as R

    return R.silu_mul(deinterleave_cols(y).to(torch.bfloat16)).float()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="8,16,32,64")
    ap.add_argument("--shapes", default="qkv,o,gate_up,down")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    ops.load()
    dev = torch.device("cuda")
    ops._sk_reserve(dev)
    torch.ops.mlop.gemm_ws_max_m(64)  # off by default in serving
    bf = torch.bfloat16
    for M in [int(m) for m in a.ms.split(",")]:
        for name in a.shapes.split(","):
            N, K = PROJ[name]
            x = torch.randn(M, K, device=dev, dtype=bf)
            ncp = max(2, (1 << 30) // (N * K * 2) + 1)
            ws = [(0.02 * torch.randn(N, K, device=dev)).to(bf) for _ in range(ncp)]
            silu = name == "gate_up"
            epi = 1 if silu else 0
            out = torch.empty(M, N // 2 if silu else N, device=dev, dtype=bf)
            cyc = [0]

            def nxt():
                cyc[0] = (cyc[0] + 1) % ncp
                return ws[cyc[0]]

            # numerics: ws vs fp32 torch
            ok = bool(torch.ops.mlop.gemm_ws(out, x, ws[0], epi, False, 0.0))
            err = None
            if ok:
                exp = x.float() @ ws[0].float().t()
                if silu:
                    exp = ref_silu_mul(exp)
                err = float((out.float() - exp).abs().max() / exp.abs().max())
            runs = {"planner": (None, lambda: ops.gemm(x, nxt(), epi=epi))}
            if ok:
                for rb in ((2, 4) if silu else (1, 2, 4)):
                    for u in (4, 8):
                        for nt in (0, 1):
                            runs[f"ws_rb{rb}_u{u}_nt{nt}"] = (
                                (rb, u, nt), lambda: torch.ops.mlop.gemm_ws(out, x, nxt(), epi, False, 0.0))
            res = {}
            for _ in range(a.rounds):
                for k, (plan, fn) in runs.items():
                    if plan is not None:
                        torch.ops.mlop.gemm_ws_plan(*plan)
                    res[k] = min(res.get(k, 1e9), timeit(fn, a.iters))
            torch.ops.mlop.gemm_ws_plan(0, 0, 1)
            best = min((k for k in res if k != "planner"), key=res.get, default=None)
            if best:
                res = {"planner": res["planner"], "ws_best": res[best], **res}
            wbytes = N * K * 2
            print(json.dumps(dict(shape=name, M=M, ws_taken=ok, rel_err=err, ws_best_plan=best if ok else None,
                                  **{f"{k}_us": round(v, 2) for k, v in res.items()},
                                  **{f"{k}_tbs": round(wbytes / v / 1e6, 2) for k, v in res.items()})), flush=True)
            del x, ws


if __name__ == "__main__":
    main()
