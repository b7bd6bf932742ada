"""MoE grouped-GEMM microbench (Mixtral-8x7B expert shapes, 8 experts, balanced routing):
one launch over all (expert, m-tile) pairs vs the same FLOPs as one dense GEMM.
Reports TFLOP/s and the expert-weight streaming rate (each expert's weights once)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlopamd import ops  # noqa: E402

ops.load()
dev = torch.device("cuda")
bf = torch.bfloat16
E, H, I = 8, 4096, 14336


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


w_gu = (0.02 * torch.randn(E, 2 * I, H, device=dev)).to(bf)
w_dn = (0.02 * torch.randn(E, H, I, device=dev)).to(bf)
for rows in [int(r) for r in os.environ.get("ROWS", "1024,2048,4096,8192").split(",")]:
    per = rows // E
    offsets = torch.arange(0, rows + 1, per, device=dev, dtype=torch.int32)[:E + 1]
    for name, w, epi, K, N in (("gate_up", w_gu, ops.EPI_SILU_MUL, H, 2 * I), ("down", w_dn, ops.EPI_NONE, I, H)):
        x = torch.randn(rows, K, device=dev, dtype=bf)
        t = min(timeit(lambda: ops.grouped_gemm(x, w, offsets, epi, avg_rows=per)) for _ in range(3))
        td = min(timeit(lambda: ops.gemm(x, w[0], epi=epi)) for _ in range(3))
        fl = 2 * rows * N * K
        print(json.dumps(dict(shape=name, rows=rows, per_expert=per, grouped_us=round(t, 1),
                              dense_same_flops_us=round(td, 1), grouped_tflops=round(fl / t / 1e6, 1),
                              weight_tbps=round(E * N * K * 2 / t / 1e6, 2))), flush=True)
