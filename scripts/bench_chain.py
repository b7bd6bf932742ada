"""Norm-chain kernels in isolation (M = 4088, Llama-3-8B gate_up / O / down shapes): plain
four-wave SiLU-mul on a normalised x vs the row-scaled (W4_RS) variant on the raw residual,
and each kernel on both inputs (is a slowdown the variant's code or the operand data?)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mlopamd import ops

torch.manual_seed(0)
dev = "cuda"
M, H, I = 4088, 4096, 14336
ops.load()
ops._sk_reserve(torch.device(dev))
res = (torch.randn(M, H, device=dev) * 4).to(torch.bfloat16)  # residual-stream magnitudes
x = ops.rmsnorm(res, torch.ones(H, device=dev, dtype=torch.bfloat16), 1e-5)
ss_res, ss_x = ops.ss_buffer(M, H, dev), ops.ss_buffer(M, H, dev)
ops.ss_parts(ss_res, M, H)[1].copy_(res.float().pow(2).sum(-1))
ops.ss_parts(ss_x, M, H)[1].copy_(x.float().pow(2).sum(-1))
wgu = (0.02 * torch.randn(2 * I, H, device=dev)).to(torch.bfloat16)
wo = (0.02 * torch.randn(H, H, device=dev)).to(torch.bfloat16)
a = torch.randn(M, H, device=dev).to(torch.bfloat16)
ss_out = ops.ss_buffer(M, H, dev)


def t(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / n


r2 = res.clone()
wd = (0.02 * torch.randn(H, I, device=dev)).to(torch.bfloat16)
act = torch.randn(M, I, device=dev).to(torch.bfloat16)
cases = {
    "gate_up silu   (x)": lambda: ops.gemm(x, wgu, epi=ops.EPI_SILU_MUL),
    "gate_up silu   (res)": lambda: ops.gemm(res, wgu, epi=ops.EPI_SILU_MUL),
    "gate_up rs     (res)": lambda: ops.gemm_rs(res, wgu, ss_res, 1e-5, ops.EPI_SILU_MUL),
    "gate_up rs     (x)": lambda: ops.gemm_rs(x, wgu, ss_x, 1e-5, ops.EPI_SILU_MUL),
    "o plain        (a)": lambda: ops.gemm(a, wo),
    "o add_ss       (a)": lambda: ops.gemm_res_ss(a, wo, r2, ss_out),
    "o + add_rmsnorm(a)": lambda: ops.add_rmsnorm(ops.gemm(a, wo), r2, torch.ones(H, device=dev, dtype=torch.bfloat16), 1e-5),
    "down plain     (act)": lambda: ops.gemm(act, wd),
    "down add_ss    (act)": lambda: ops.gemm_res_ss(act, wd, r2, ss_out),
}
for rnd in range(3):
    print("round", rnd, "  ".join(f"{k}: {t(f):7.1f}" for k, f in cases.items()), flush=True)
flops = {"gate_up": 2 * M * 2 * I * H, "o": 2 * M * H * H, "down": 2 * M * H * I}
for k, f in cases.items():
    us = min(t(f) for _ in range(2))
    print(f"{k:22s} {us:8.1f} us  {flops[k.split()[0]] / us / 1e9:7.1f} TF/s", flush=True)
