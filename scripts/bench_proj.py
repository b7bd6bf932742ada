"""Op-level A/B of the projection alternatives the autotuner picks between, at the
headline's row counts (Llama-3-8B, random data, one process, interleaved rounds):

  qkv      fused QKV GEMM + RoPE + paged K/V stores (EPI_ROPE)  vs  hipBLASLt + rope_cache
  gate_up  MFMA GEMM with the SiLU-mul epilogue                 vs  hipBLASLt + silu_mul
  o, down  MFMA GEMM (split-K reduce does add + RMSNorm)        vs  hipBLASLt + add_rmsnorm

BENCH_MS = comma list of M (default: decode-only and mixed-step sizes of the bench)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlopamd import ops  # noqa: E402
from mlopamd.models.layers import rope_table  # noqa: E402

ops.load()
dev = torch.device("cuda")
bf = torch.bfloat16
Ms = [int(m) for m in os.environ.get("BENCH_MS", "2040,2048,2304,3072,4088,4352,6144,8192").split(",")]
CUR_M = 0
H, I, D, Hq, Hkv, BS = 4096, 14336, 128, 32, 8, 16


COLD_M = int(os.environ.get("COLD_M", "256"))  # at or below: weights stream from HBM each step
_flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)


def timeit_cold(fn, iters=10):
    """Per-call time with L2 + the 256 MB MALL evicted before every call (decode reads each
    weight once per step, cold)."""
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    tot = 0.0
    for _ in range(iters):
        _flush.fill_(1)
        s.record()
        fn()
        e.record()
        e.synchronize()
        tot += s.elapsed_time(e)
    return tot / iters * 1e3


def timeit(fn, iters=20):
    if CUR_M <= COLD_M:
        return timeit_cold(fn)
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


def forced(backend, fn):
    def run():
        ops.GEMM_BACKEND = backend
        try:
            return fn()
        finally:
            ops.GEMM_BACKEND = ops.GEMM_BACKEND_DEFAULT
    return run


cs = rope_table(D, 8192, 5e5, device=dev)
w_qkv = (0.02 * torch.randn((Hq + 2 * Hkv) * D, H, device=dev)).to(bf)
w_o = (0.02 * torch.randn(H, H, device=dev)).to(bf)
w_gu = (0.02 * torch.randn(2 * I, H, device=dev)).to(bf)
w_dn = (0.02 * torch.randn(H, I, device=dev)).to(bf)
nw = torch.ones(H, device=dev, dtype=bf)
for M in Ms:
    CUR_M = M
    NB = M // BS + 8
    x = torch.randn(M, H, device=dev, dtype=bf)
    xi = torch.randn(M, I, device=dev, dtype=bf)
    res = torch.randn(M, H, device=dev, dtype=bf)
    pos = torch.randint(0, 8000, (M,), device=dev, dtype=torch.int32)
    slots = torch.randperm(NB * BS, device=dev)[:M].to(torch.int32)
    kc = torch.zeros(NB, Hkv, BS, D, device=dev, dtype=bf)
    vc = torch.zeros(NB, Hkv, BS, D, device=dev, dtype=bf)
    cases = {
        "qkv": lambda: ops.qkv_rope_cache(x, w_qkv, pos, cs, slots, kc, vc, Hq),
        "gate_up": lambda: ops.gemm(x, w_gu, epi=ops.EPI_SILU_MUL),
        "o": lambda: ops.gemm_add_rmsnorm(x, w_o, res, nw, 1e-5),
        "down": lambda: ops.gemm_add_rmsnorm(xi, w_dn, res, nw, 1e-5),
    }
    for name, fn in cases.items():
        tm, th = [], []
        for _ in range(3):
            tm.append(timeit(forced("mlop", fn)))
            th.append(timeit(forced("hipblaslt", fn)))
        a, b = min(tm), min(th)
        print(json.dumps(dict(shape=name, M=M, mlop_us=round(a, 1), hipblaslt_us=round(b, 1),
                              winner="mlop" if a < b else "hipblaslt", margin=round(max(a, b) / min(a, b) - 1, 3))),
              flush=True)
