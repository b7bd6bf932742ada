"""Run one GEMM shape repeatedly (for rocprofv3 counter collection).
env: SHAPE=M,N,K  EPI=0|1|3  ITERS=n  BACKEND=mlop|hipblaslt  BIG_VARIANT=3|4 (large-M kernel)
EPI=3: the fused QKV projection (RoPE + paged K + V staging; N = (Hq + 2 Hkv) * 128, Hkv = 8)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlopamd import ops  # noqa: E402

ops.load()
M, N, K = (int(v) for v in os.environ.get("SHAPE", "8192,6144,4096").split(","))
epi = int(os.environ.get("EPI", "0"))
iters = int(os.environ.get("ITERS", "20"))
be = os.environ.get("BACKEND", "mlop")
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = (0.02 * torch.randn(N, K, device="cuda")).to(torch.bfloat16)
ops.GEMM_BACKEND = "mlop"
if os.environ.get("BIG_VARIANT"):
    torch.ops.mlop.gemm_big_variant(int(os.environ["BIG_VARIANT"]))
if epi == 3:
    from mlopamd.models.layers import rope_table

    Hkv, D, BS = 8, 128, 16
    Hq = N // D - 2 * Hkv
    NB = M // BS + 8
    cs = rope_table(D, 8192, 5e5, device="cuda")
    pos = torch.randint(0, 8000, (M,), device="cuda", dtype=torch.int32)
    slots = torch.randperm(NB * BS, device="cuda")[:M].to(torch.int32)
    kc = torch.zeros(NB, Hkv, BS, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.zeros(NB, Hkv, BS, D, device="cuda", dtype=torch.bfloat16)
for _ in range(iters):
    if be == "mlop" and epi == 3:
        ops.qkv_rope_cache(x, w, pos, cs, slots, kc, vc, Hq)
    elif be == "mlop":
        ops.gemm(x, w, epi=epi)
    else:
        torch.matmul(x, w.t())
torch.cuda.synchronize()
print("done", M, N, K, be)
