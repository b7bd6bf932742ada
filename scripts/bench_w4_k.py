"""Per-K-tile cost vs fixed per-tile cost of the large-M GEMM kernels: time(K) at
M = N = 4096 (256 tiles = one per CU) for K = 1024 .. 16384, and at N = 28672 (7 tiles per
CU).  A least-squares line t = a + b * (K / 64) gives b = one K-tile's time and a = the
prologue + epilogue of a tile (per tile wave).  Variants: 3 ping-pong, 5 four-wave; hipBLASLt
for reference.  One process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlopamd import ops  # noqa: E402

ops.load()
dev = torch.device("cuda")
ops.GEMM_BACKEND = "mlop"
Vs = [int(v) for v in os.environ.get("BENCH_VARIANTS", "3,5").split(",")]


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


for M, N in ((4096, 4096), (4096, 28672)):
    Ks = [1024, 2048, 4096, 8192, 16384] if N == 4096 else [1024, 2048, 4096, 8192]
    res = {}
    for K in Ks:
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = (0.02 * torch.randn(N, K, device=dev)).to(torch.bfloat16)
        cands = {}
        for v in Vs:
            def f(v=v):
                torch.ops.mlop.gemm_big_variant(v)
                return ops.gemm(x, w)
            cands[f"v{v}"] = f
        cands["hipblaslt"] = lambda: torch.matmul(x, w.t())
        ts = {k: min(timeit(f) for _ in range(3)) for k, f in cands.items()}
        res[K] = ts
        print(json.dumps({"M": M, "N": N, "K": K, **{k: round(v, 1) for k, v in ts.items()}}), flush=True)
    for k in res[Ks[0]]:
        xs = np.array([K / 64 for K in Ks])
        ys = np.array([res[K][k] for K in Ks])
        b, a = np.polyfit(xs, ys, 1)
        print(json.dumps({"M": M, "N": N, "kernel": k, "us_per_ktile": round(b, 3), "fixed_us": round(a, 2)}), flush=True)
torch.ops.mlop.gemm_big_variant(5)
