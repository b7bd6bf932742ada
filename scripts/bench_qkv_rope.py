"""QKV projection + RoPE + paged-KV write: the fused MFMA epilogue (EPI_ROPE) vs
hipBLASLt GEMM + rope_cache kernel, Llama-3-8B shapes, random data (one process,
interleaved rounds, min of 3)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlopamd import ops  # noqa: E402
from mlopamd.models.layers import rope_table  # noqa: E402

ops.load()
dev = torch.device("cuda")
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


# SLAB_NT: gemm_slab_nt values to interleave (e.g. "15,7": bit 3 = the RoPE epilogue's q / K / V
# stores non-temporal)
NTS = [int(v) for v in os.environ.get("SLAB_NT", str(torch.ops.mlop.gemm_slab_nt(-1))).split(",")]
for M, nt in [(int(m), nt) for m in os.environ.get("BENCH_MS", "512,1024,2048,3072,4096").split(",") for nt in NTS]:
    torch.ops.mlop.gemm_slab_nt(nt)
    NB = M // BS + 8
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    pos = torch.randint(0, 8000, (M,), device=dev, dtype=torch.int32)
    slots = torch.randperm(NB * BS, device=dev)[:M].to(torch.int32)
    kc = torch.zeros(NB, Hkv, BS, D, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros(NB, Hkv, BS, D, device=dev, dtype=torch.bfloat16)
    q = torch.empty(M, Hq, D, device=dev, dtype=torch.bfloat16)
    fused = lambda: torch.ops.mlop.gemm_rope_cache(q, kc, vc, x, w, pos, cs, slots)  # noqa: E731
    unf = lambda: ops.rope_cache(torch.matmul(x, w.t()), pos, cs, slots, kc, vc, Hq, q)  # noqa: E731
    rope_only_in = torch.matmul(x, w.t())
    rope = lambda: ops.rope_cache(rope_only_in, pos, cs, slots, kc, vc, Hq, q)  # noqa: E731
    noslot = torch.full_like(slots, -1)
    fused_ns = lambda: torch.ops.mlop.gemm_rope_cache(q, kc, vc, x, w, pos, cs, noslot)  # noqa: E731
    plain = lambda: ops._gemm_mlop(x, w, torch.empty(M, N, device=dev, dtype=torch.bfloat16), 0)  # noqa: E731
    tf, tu, tr, tn, tp = [], [], [], [], []
    for _ in range(3):
        tf.append(timeit(fused))
        tu.append(timeit(unf))
        tr.append(timeit(rope))
        tn.append(timeit(fused_ns))
        tp.append(timeit(plain))
    print(json.dumps(dict(M=M, slab_nt=nt, fused_us=round(min(tf), 1), hipblaslt_plus_rope_us=round(min(tu), 1),
                          rope_cache_us=round(min(tr), 1), fused_noslots_us=round(min(tn), 1),
                          mlop_plain_us=round(min(tp), 1), speedup=round(min(tu) / min(tf), 2),
                          fused_tflops=round(2 * M * N * K / min(tf) / 1e6, 1))), flush=True)
