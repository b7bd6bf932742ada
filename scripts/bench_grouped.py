"""MoE grouped GEMM A/B at Mixtral-8x7B sizes (8 experts, ~T*2/8 routed rows each): the
ping-pong kernel with the stream-K tail on vs off (gemm_sk_mode), gate_up (SiLU epilogue,
N=28672, K=4096) and down (N=4096, K=14336).  ROWS = routed rows in total."""
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
rng = np.random.default_rng(0)
E = 8


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


ops._sk_reserve(dev)
for rows in [int(r) for r in os.environ.get("ROWS", "2048,4088,8176").split(",")]:
    counts = rng.multinomial(rows, [1 / E] * E)
    off = torch.tensor([0] + list(np.cumsum(counts)), device=dev, dtype=torch.int32)
    for name, N, K, epi in (("gate_up", 28672, 4096, 1), ("down", 4096, 14336, 0)):
        x = torch.randn(rows, K, device=dev, dtype=bf)
        w = (0.02 * torch.randn(E, N, K, device=dev)).to(bf)
        res = {}
        for _ in range(2):  # interleaved rounds
            for mode in (1, 0):
                torch.ops.mlop.gemm_sk_mode(mode)
                t = timeit(lambda: ops.grouped_gemm(x, w, off, epi=epi, avg_rows=rows // E))
                res[mode] = min(res.get(mode, 1e9), t)
        torch.ops.mlop.gemm_sk_mode(1)
        flops = 2 * rows * N * K
        print(json.dumps(dict(shape=name, rows=rows, counts=counts.tolist(), sk_us=round(res[1], 1),
                              dp_us=round(res[0], 1), sk_tflops=round(flops / res[1] / 1e6, 1))), flush=True)
        del x, w
