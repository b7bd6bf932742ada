"""A/B of the large-M GEMM at the headline's row counts (Llama-3-8B projections, random data,
one process, interleaved rounds; cdna_hip_programming.md §5.4 rule 24): the ping-pong 8-wave
256x256 kernel (gemm.hip, planner variant 3) vs hipBLASLt (torch.matmul).  Plain GEMMs
(epilogue-free) except gate_up, which the hand-written kernel runs with the fused SiLU-mul
epilogue (hipBLASLt without it).  Env: BENCH_MS (comma list of row counts), BENCH_VARIANTS
(planner variants of the hand-written kernel: 3 ping-pong, 5 four-wave asm loop)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlopamd import ops  # noqa: E402

ops.load()
dev = torch.device("cuda")
Ms = [int(m) for m in os.environ.get("BENCH_MS", "2048,4088").split(",")]
Vs = [int(v) for v in os.environ.get("BENCH_VARIANTS", "3").split(",")]
ops._sk_reserve(dev)
ops.GEMM_BACKEND = "mlop"


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
    return s.elapsed_time(e) / iters * 1e3


def with_variant(v, fn):
    def run():
        torch.ops.mlop.gemm_big_variant(v)
        return fn()
    return run


for M in Ms:
    for name, N, K in (("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)):
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = (0.02 * torch.randn(N, K, device=dev)).to(torch.bfloat16)
        epi = ops.EPI_SILU_MUL if name == "gate_up" else ops.EPI_NONE
        cands = {f"v{v}": with_variant(v, lambda: ops.gemm(x, w, epi=epi)) for v in Vs}
        cands["hipblaslt"] = lambda: torch.matmul(x, w.t())
        ts = {k: [] for k in cands}
        for _ in range(3):
            for k, f in cands.items():
                ts[k].append(timeit(f))
        best = {k: round(min(v), 1) for k, v in ts.items()}
        fl = 2 * M * N * K
        print(json.dumps(dict(shape=name, M=M, N=N, K=K, **{f"{k}_us": v for k, v in best.items()},
                              **{f"{k}_tflops": round(fl / v / 1e6) for k, v in best.items()})), flush=True)
torch.ops.mlop.gemm_big_variant(3)
