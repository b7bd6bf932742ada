"""Does a per-shape library-solution search beat torch.matmul's default hipBLASLt pick?

For each Llama-3-8B projection shape at the headline's row counts: time torch.matmul
(default heuristic solution), then let PyTorch's TunableOp benchmark every hipBLASLt /
rocBLAS solution for that exact (M, N, K), and time again with the chosen solution.
The hand-written ping-pong kernel is timed alongside for reference.  Interleaved rounds,
min of 3, random data, one process."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlopamd import ops  # noqa: E402

ops.load()
dev = torch.device("cuda")
Ms = [int(m) for m in os.environ.get("BENCH_MS", "2048,3072,4096").split(",")]
out_csv = os.environ.get("TUNABLE_CSV", "gpurun_out/tunableop_results.csv")
shapes = [(n, M, N, K) for M in Ms for n, N, K in (("qkv", 6144, 4096), ("o", 4096, 4096),
                                                     ("gate_up", 28672, 4096), ("down", 4096, 14336))]


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


def mlop(x, w):
    ops.GEMM_BACKEND = "mlop"
    try:
        return ops.gemm(x, w, epi=ops.EPI_NONE)
    finally:
        ops.GEMM_BACKEND = ops.GEMM_BACKEND_DEFAULT


tun = torch.cuda.tunable
data = []
for name, M, N, K in shapes:
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = (0.02 * torch.randn(N, K, device=dev)).to(torch.bfloat16)
    data.append((name, M, N, K, x, w))

tun.enable(False)
base = {}
for name, M, N, K, x, w in data:
    base[(name, M)] = (min(timeit(lambda: torch.matmul(x, w.t())) for _ in range(3)),
                       min(timeit(lambda: mlop(x, w)) for _ in range(3)))
    print("base", name, M, base[(name, M)], flush=True)

tun.enable(True)
tun.tuning_enable(True)
tun.set_max_tuning_duration(100)
tun.set_max_tuning_iterations(20)
tun.set_filename(out_csv)
for name, M, N, K, x, w in data:
    torch.matmul(x, w.t())  # tunes this shape
    torch.cuda.synchronize()
    print("tuned", name, M, flush=True)
tun.tuning_enable(False)
for name, M, N, K, x, w in data:
    tt = min(timeit(lambda: torch.matmul(x, w.t())) for _ in range(3))
    td, tm = base[(name, M)]
    f = 2 * M * N * K
    print(json.dumps(dict(shape=name, M=M, N=N, K=K, default_us=round(td, 1), tuned_us=round(tt, 1),
                          mlop_us=round(tm, 1), default_tf=round(f / td / 1e6), tuned_tf=round(f / tt / 1e6),
                          mlop_tf=round(f / tm / 1e6), tuned_vs_default=round(td / tt, 3))), flush=True)
tun.write_file(out_csv)
print("results", tun.get_results())
