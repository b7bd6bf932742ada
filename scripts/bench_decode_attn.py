"""Decode paged-attention microbench (Llama-3-8B heads: 32 q / 8 kv, D=128, pages of 16
tokens scattered over the pool): B sequences x 1 query token at context L.  Reports
the KV bytes streamed per call and the effective HBM rate (roofline ~6.3 TB/s)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from mlopamd import ops  # noqa: E402
from mlopamd.runtime.attn_meta import plan_partitions  # noqa: E402
from test_kernels_gpu import make_meta  # noqa: E402

ops.load()
dev = torch.device("cuda")
bf = torch.bfloat16
Hq, Hkv, D = 32, 8, 128


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


cases = [(int(b), int(l)) for b, l in (c.split("x") for c in
                                       os.environ.get("CASES", "2048x384,1024x384,256x1024,64x4096,8x8192").split(","))]
for B, L in cases:
    np.random.seed(0)
    ctx = np.random.randint(max(16, L // 2), L * 3 // 2 + 1, size=B).tolist()
    NB = sum((c + 15) // 16 for c in ctx) + 8
    kc = torch.randn(NB, Hkv, 16, D, device=dev, dtype=bf)
    vc = torch.randn(NB, Hkv, 16, D, device=dev, dtype=bf)
    m, T = make_meta(dev, [1] * B, ctx, Hkv, Hq // Hkv, NB)
    nparts = m.nparts
    q = torch.randn(T, Hq, D, device=dev, dtype=bf)
    t = min(timeit(lambda: ops.paged_attention(q, kc, vc, m)) for _ in range(3))
    byts = sum(ctx) * Hkv * D * 2 * 2
    print(json.dumps(dict(B=B, mean_ctx=round(float(np.mean(ctx)), 1), nparts=nparts, us=round(t, 1),
                          kv_gb=round(byts / 1e9, 3), tbps=round(byts / t / 1e6, 2))), flush=True)
