"""add + RMSNorm / RMSNorm at the headline's row counts (Llama-3-8B hidden 4096): us per call
and the implied bytes/s (x, residual read + written, out written; weight from L2).  Measured
2026-10-17 (scripts/r3b_norm.sh): add + RMSNorm 19.9 us at M = 4088 = 6.7 TB/s, RMSNorm 10.9 us
= 6.1 TB/s, i.e. at the HBM roof; loading the weight with the row (one round trip instead of
two) changed nothing (19.85 vs 19.93 us) and was not kept."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlopamd import ops  # noqa: E402

if os.environ.get("NORM_LIB"):  # A/B against another build of the extension (same op names)
    torch.ops.load_library(os.environ["NORM_LIB"])
else:
    ops.load()
dev = torch.device("cuda")


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


H = 4096
for M in (4088, 2048):
    x = torch.randn(M, H, device=dev, dtype=torch.bfloat16)
    r = torch.randn(M, H, device=dev, dtype=torch.bfloat16)
    w = torch.randn(H, device=dev, dtype=torch.bfloat16)
    out = torch.empty_like(x)
    t_add = min(timeit(lambda: torch.ops.mlop.add_rmsnorm(out, r, x, w, 1e-5)) for _ in range(3))
    t_n = min(timeit(lambda: torch.ops.mlop.rmsnorm(out, x, w, 1e-5)) for _ in range(3))
    print(json.dumps({"lib": os.environ.get("NORM_LIB", "tree"), "M": M, "add_rmsnorm_us": round(t_add, 2), "add_TBps": round(4 * M * H * 2 / t_add / 1e6, 2),
                      "rmsnorm_us": round(t_n, 2), "rms_TBps": round(2 * M * H * 2 / t_n / 1e6, 2)}), flush=True)
