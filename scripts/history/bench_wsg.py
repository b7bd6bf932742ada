"""Mid-size decode projections (M = 8..64): wsgemm.hip (register-streamed MFMA) vs the
LDS-DMA MFMA tiles (gemm.hip, wsgemm off) vs hipBLASLt, Llama-3-8B shapes.

Decode reads every weight once per step, so the weights rotate over enough copies (> 1 GB)
that no call finds its matrix in L2 / the 256 MB MALL; us per call over one pass of the copies,
best of 3 interleaved rounds (cdna_hip_programming.md §5.4 rule 24).  TB/s = weight bytes / time.
Env: BENCH_MS (row counts), WSG_MIN_WG (comma list swept for the wsgemm arm, empty = none),
SMALL_TILES (gemm_small_tile values: row-fitted BM x 32 / 64 LDS-DMA tiles)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlopamd import ops  # noqa: E402

ops.load()
dev = torch.device("cuda")
Ms = [int(m) for m in os.environ.get("BENCH_MS", "8,16,32,64").split(",")]
MIN_WG = [int(v) for v in os.environ.get("WSG_MIN_WG", "256").split(",") if v]
SMALL_TILES = [int(v) for v in os.environ.get("SMALL_TILES", "").split(",") if v]  # gemm_small_tile arms
STAGES = [int(v) for v in os.environ.get("SMALL_STAGES", "3").split(",") if v]  # gemm_small_stages sweep
SHAPES = (("qkv", 6144, 4096, 0), ("o", 4096, 4096, 2), ("gate_up", 28672, 4096, 1), ("down", 4096, 14336, 2))


def run_pass(fn, ws, xs):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn(ws[0], xs[0])
    torch.cuda.synchronize()
    s.record()
    for i, w in enumerate(ws):
        fn(w, xs[i % len(xs)])
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / len(ws)


for name, N, K, epi in SHAPES:
    copies = max(4, (1 << 30) // (N * K * 2) + 1)
    ws = [(0.02 * torch.randn(N, K, device=dev)).to(torch.bfloat16) for _ in range(copies)]
    for M in Ms:
        xs = [torch.randn(M, K, device=dev, dtype=torch.bfloat16) for _ in range(2)]
        res = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        nw = torch.ones(N, device=dev, dtype=torch.bfloat16)
        gepi = 1 if epi == 1 else 0
        out = torch.empty(M, N // 2 if gepi else N, device=dev, dtype=torch.bfloat16)

        def mlop(w, x):
            if epi == 2:
                ops.GEMM_BACKEND = "mlop"
                try:
                    ops.gemm_add_rmsnorm(x, w, res, nw, 1e-5)
                finally:
                    ops.GEMM_BACKEND = "auto"
            else:
                nws = torch.ops.mlop.gemm_workspace(M, N, K, gepi)
                torch.ops.mlop.gemm(out, x, w, torch.empty(max(nws, 1), device=dev), gepi)

        def blas(w, x):
            y = torch.matmul(x, w.t())
            if epi == 1:
                torch.ops.mlop.silu_mul(out, y, 1)
            elif epi == 2:
                ops.add_rmsnorm(y, res, nw, 1e-5)

        arms = {}
        for r in range(3):
            torch.ops.mlop.gemm_wsg_config(0, 256)
            arms["tiles"] = min(arms.get("tiles", 1e9), run_pass(mlop, ws, xs))
            for mw in MIN_WG:
                torch.ops.mlop.gemm_wsg_config(64, mw)
                k = f"wsg{mw}"
                arms[k] = min(arms.get(k, 1e9), run_pass(mlop, ws, xs))
            for st in SMALL_TILES:
                torch.ops.mlop.gemm_small_tile(st)
                for sg in STAGES:
                    torch.ops.mlop.gemm_small_stages(sg)
                    k = f"st{st}" + (f"s{sg}" if len(STAGES) > 1 else "")
                    arms[k] = min(arms.get(k, 1e9), run_pass(mlop, ws, xs))
                torch.ops.mlop.gemm_small_stages(3)
            torch.ops.mlop.gemm_small_tile(0)
            arms["hipblaslt"] = min(arms.get("hipblaslt", 1e9), run_pass(blas, ws, xs))
        torch.ops.mlop.gemm_wsg_config(0, 256)
        wb = N * K * 2
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "epi": ["none", "silu", "add_rmsnorm"][epi],
                          **{f"{k}_us": round(v, 1) for k, v in arms.items()},
                          **{f"{k}_tbps": round(wb / v / 1e6, 2) for k, v in arms.items()}}), flush=True)
    del ws
    torch.cuda.empty_cache()
