"""Fused QKV + RoPE + paged-KV GEMM (EPI_ROPE) on the large-M kernels: planner variant 3
(ping-pong, 512 threads, stream-K tail) vs 5 (four-wave asm loop, K-half tail), plus the plain
QKV GEMM of each for the epilogue's share.  One process, interleaved rounds, min of 3."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlopamd import ops  # noqa: E402
from mlopamd.models.layers import rope_table  # noqa: E402

ops.load()
dev = torch.device("cuda")
ops._sk_reserve(dev)
ops.GEMM_BACKEND = "mlop"
Hq, Hkv, D, K, BS = 32, 8, 128, 4096, 16
N = (Hq + 2 * Hkv) * D
cs = rope_table(D, 8192, 5e5, device=dev)
w = (0.02 * torch.randn(N, K, device=dev)).to(torch.bfloat16)


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


for M in [int(m) for m in os.environ.get("BENCH_MS", "4088,2048").split(",")]:
    NB = M // BS + 8
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    pos = torch.randint(0, 8000, (M,), device=dev, dtype=torch.int32)
    slots = torch.randperm(NB * BS, device=dev)[:M].to(torch.int32)
    kc = torch.zeros(NB, Hkv, BS, D, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros(NB, Hkv, BS, D, device=dev, dtype=torch.bfloat16)
    q = torch.empty(M, Hq, D, device=dev, dtype=torch.bfloat16)
    res = {}
    for _ in range(3):
        for v in (3, 5):
            torch.ops.mlop.gemm_big_variant(v)
            t = timeit(lambda: torch.ops.mlop.gemm_rope_cache(q, kc, vc, x, w, pos, cs, slots))
            res[f"rope_v{v}"] = min(res.get(f"rope_v{v}", 1e9), t)
            t = timeit(lambda: ops.gemm(x, w))
            res[f"plain_v{v}"] = min(res.get(f"plain_v{v}", 1e9), t)
        torch.ops.mlop.gemm_big_variant(5)
        qkv = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        t = timeit(lambda: (ops._gemm_mlop(x, w, qkv, 0), ops.rope_cache(qkv, pos, cs, slots, kc, vc, Hq, q)))
        res["unfused_v5"] = min(res.get("unfused_v5", 1e9), t)
        t = timeit(lambda: ops.rope_cache(qkv, pos, cs, slots, kc, vc, Hq, q))
        res["rope_cache_only"] = min(res.get("rope_cache_only", 1e9), t)
    torch.ops.mlop.gemm_big_variant(5)
    print(json.dumps({"M": M, "v_stage": os.environ.get("MLOP_V_STAGE", "1"),
                      **{k: round(v, 1) for k, v in res.items()}}), flush=True)
