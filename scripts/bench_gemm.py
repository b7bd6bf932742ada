"""GEMM microbench on the Llama-3-8B (or BENCH_MODEL=70b: Llama-3-70B) projection shapes: the hand-written MFMA
GEMM (forced, ``ops.GEMM_BACKEND = "mlop"``) vs torch.matmul (hipBLASLt).
One process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24), random data.
Individual tilings are forced with ``torch.ops.mlop.gemm_dense_plan`` (scripts/bench_mid_m.py)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlopamd import ops  # noqa: E402

ops.load()
dev = torch.device("cuda")
Ms = [int(m) for m in os.environ.get("BENCH_MS", "1,64,128,256,512,8192").split(",")]
PROJ = {"8b": (("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096),
                ("down", 4096, 14336), ("lm_head", 128256, 4096)),
        "70b": (("qkv", 10240, 8192), ("o", 8192, 8192), ("gate_up", 57344, 8192),
                ("down", 8192, 28672), ("lm_head", 128256, 8192))}[os.environ.get("BENCH_MODEL", "8b")]
shapes = []
for M in Ms:
    for name, N, K in PROJ:
        if name == "lm_head" and M > 512:
            continue
        shapes.append((name, M, N, K))


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def mlop(x, w, epi):
    ops.GEMM_BACKEND = "mlop"
    try:
        return ops.gemm(x, w, epi=epi)
    finally:
        ops.GEMM_BACKEND = ops.GEMM_BACKEND_DEFAULT


tag = os.environ.get("BENCH_TAG", "")
for name, M, N, K in shapes:
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = (0.02 * torch.randn(N, K, device=dev)).to(torch.bfloat16)
    epi = ops.EPI_SILU_MUL if name == "gate_up" else ops.EPI_NONE
    ts_m, ts_t = [], []
    for _ in range(3):
        ts_m.append(timeit(lambda: mlop(x, w, epi)))
        ts_t.append(timeit(lambda: torch.matmul(x, w.t())))
    tm, tt = min(ts_m), min(ts_t)
    flops = 2 * M * N * K
    byts = 2 * (N * K + M * K + M * N)
    print(json.dumps(dict(tag=tag, shape=name, M=M, N=N, K=K, mlop_us=round(tm, 1), hipblaslt_us=round(tt, 1),
                          mlop_tflops=round(flops / tm / 1e6, 1), mlop_tbps=round(byts / tm / 1e6, 2),
                          speedup=round(tt / tm, 2))), flush=True)
