"""Does a decode GEMV read its weights faster right after they were pulled into the 256 MiB
Infinity Cache?  Batch-1 Llama-3-8B shapes: o (4096 x 4096), qkv (6144 x 4096), down
(4096 x 14336).  Per shape, each timed with events, median of 20:
  cold      : a 1 GiB buffer is read first (evicts the weights), then the GEMV;
  prefetched: the same flush, then one read pass over the weight (a sum kernel), then the GEMV.
Only the GEMV is inside the events.  If 'prefetched' is much shorter, streaming the next
projection's weights during the latency-bound attention / norm launches of the decode step
would shorten that projection."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlopamd import ops  # noqa: E402

ops.load()
dev = torch.device("cuda")
bf = torch.bfloat16
flush = torch.empty(1 << 29, dtype=bf, device=dev)  # 1 GiB
flush.fill_(1.0)
x = torch.randn(1, 4096, device=dev, dtype=bf)
for name, N, K in (("o", 4096, 4096), ("qkv", 6144, 4096), ("down", 4096, 14336), ("gate_up", 28672, 4096)):
    w = (0.02 * torch.randn(N, K, device=dev)).to(bf)
    xk = torch.randn(1, K, device=dev, dtype=bf)
    res = {}
    for mode in ("cold", "prefetched", "cold", "prefetched"):
        ts = []
        for _ in range(20):
            flush.sum()
            if mode == "prefetched":
                w.view(-1).sum()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.gemm(xk, w)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        res.setdefault(mode, []).append(round(ts[len(ts) // 2], 1))
    mb = N * K * 2 / 1e6
    print(json.dumps(dict(shape=name, weight_mb=round(mb, 1), cold_us=res["cold"], prefetched_us=res["prefetched"],
                          cold_tbps=round(mb / min(res["cold"]), 2), prefetched_tbps=round(mb / min(res["prefetched"]), 2))),
          flush=True)
