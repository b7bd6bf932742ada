"""Run one GEMM shape repeatedly (for rocprofv3 counter collection).
env: SHAPE=M,N,K  EPI=0|1  ITERS=n  BACKEND=mlop|hipblaslt  BIG_VARIANT=3|4 (large-M kernel)"""
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
for _ in range(iters):
    if be == "mlop":
        ops.gemm(x, w, epi=epi)
    else:
        torch.matmul(x, w.t())
torch.cuda.synchronize()
print("done", M, N, K, be)
