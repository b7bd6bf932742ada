"""Race screens for the cross-workgroup hand-off protocols, under uneven load.

Three kernels hand work between workgroups of ONE launch through global memory, with
no assumption on dispatch order or co-residency (MI355X_MICROARCH.md "Correctness
boundaries"):

  * the ping-pong GEMM's stream-K tail: sc1 write-through fp32 partial slots, an
    agent-scope ticket per tail tile, the last contributor sums the slots and re-arms
    the counter (ops/csrc/gemm.hip ``gemm_pp_kernel<.., SK=true>``);
  * the grouped (MoE) GEMM, whose stream-K split is planned ON DEVICE from the routed
    offsets;
  * paged attention's fused split-KV combine: the last-arriving partition of a
    (tile, kv head) merges the partial softmax slabs and re-arms its semaphore
    (ops/csrc/attention.hip).

A protocol bug (a read placed before the release it depends on, a counter that is not
re-armed) shows up as a result that changes from launch to launch, mostly when workgroups
arrive in an unusual order.  Each test therefore launches the kernel many times while a
second HIP stream keeps a large GEMM running (it occupies CUs for unpredictable stretches,
so the protocol kernel's workgroups are placed and delayed unevenly), and requires every
result to be BIT-identical to a quiet reference launch (the fixup sums in a fixed slot
order, so the result is deterministic) and close to the fp32 oracle.  Test strategy:
SURVEY.md §5 "race detection" (GPU side: flag-protocol tests under uneven load); the
custom all-reduce's epoch flags get the same treatment across processes in
test_custom_ar_gpu.py.
"""
import numpy as np
import pytest
import torch

from mlopamd import ops
from mlopamd.ops import reference as ref

pytestmark = pytest.mark.gpu
bf = torch.bfloat16
REPS = 24


class _Noise:
    """A side stream that keeps a big bf16 GEMM in flight (queued ahead of each launch)."""

    def __init__(self, dev):
        self.s = torch.cuda.Stream(device=dev)
        self.a = torch.randn(4096, 4096, device=dev, dtype=bf)
        self.b = torch.randn(4096, 4096, device=dev, dtype=bf)
        self.c = torch.empty(4096, 4096, device=dev, dtype=bf)

    def kick(self, n=2):
        with torch.cuda.stream(self.s):
            for _ in range(n):
                torch.matmul(self.a, self.b, out=self.c)

    def drain(self):
        self.s.synchronize()


def _under_contention(dev, launch, reps=REPS):
    """Quiet reference launch, then ``reps`` launches each racing a noise GEMM whose
    amount varies per launch; returns (reference, list of mismatching launch indices)."""
    ref_out = launch().clone()
    torch.cuda.synchronize()
    noise = _Noise(dev)
    bad = []
    for i in range(reps):
        noise.kick(1 + i % 3)
        y = launch()
        if not torch.equal(y, ref_out):
            bad.append(i)
    noise.drain()
    torch.cuda.synchronize()
    return ref_out, bad


@pytest.mark.parametrize("M,N,K,epi", [
    (2040, 28672, 4096, 1),   # 128 tail tiles in 2 halves, SiLU-mul epilogue in the fixup
    (4352, 4096, 14336, 0),   # 16 tail tiles x 8 ranges (the re-read sum path)
    (3072, 6144, 4096, 0),
])
def test_stream_k_tickets_under_contention(gpu, pp_variant, M, N, K, epi):
    torch.manual_seed(M)
    ops._sk_reserve(torch.device(gpu))
    assert torch.ops.mlop.gemm_sk_workgroups(M, N, K) > 0, "shape must take the stream-K tail"
    x = torch.randn(M, K, device=gpu, dtype=bf)
    w = (0.05 * torch.randn(N, K, device=gpu)).to(bf)
    ops.GEMM_BACKEND = "mlop"
    try:
        y0, bad = _under_contention(gpu, lambda: ops.gemm(x, w, epi=epi))
    finally:
        ops.GEMM_BACKEND = ops.GEMM_BACKEND_DEFAULT
    assert not bad, f"stream-K result changed on launches {bad}"
    exp = x.float() @ w.float().t()
    if epi:
        exp = ref.silu_mul(ops.deinterleave_cols(exp.to(bf)))
    tol = 3e-2 * exp.abs().max().item() / 10 + 1e-2
    torch.testing.assert_close(y0.float(), exp.float(), atol=tol, rtol=2e-2)


@pytest.mark.parametrize("counts,epi,N,K", [
    ([530, 498, 512, 470, 555, 505, 490, 528], 0, 4096, 14336),
    ([16, 17, 15, 16, 16, 18, 14, 16], 1, 28672, 4096),   # split-K grouped + reduce
])
def test_grouped_stream_k_under_contention(gpu, counts, epi, N, K):
    torch.manual_seed(sum(counts))
    ops._sk_reserve(torch.device(gpu))
    E = len(counts)
    off = torch.tensor([0] + list(np.cumsum(counts)), device=gpu, dtype=torch.int32)
    Mt = int(off[-1])
    x = torch.randn(Mt, K, device=gpu, dtype=bf)
    w = (0.02 * torch.randn(E, N, K, device=gpu)).to(bf)
    y0, bad = _under_contention(gpu, lambda: ops.grouped_gemm(x, w, off, epi=epi, avg_rows=Mt // E))
    assert not bad, f"grouped stream-K result changed on launches {bad}"
    for e in (0, E - 1):
        a, b = int(off[e]), int(off[e + 1])
        r = x[a:b].float() @ w[e].float().t()
        if epi:
            r = ref.silu_mul(ops.deinterleave_cols(r.to(bf)))
        torch.testing.assert_close(y0[a:b].float(), r.float(), atol=3e-2, rtol=3e-2)


def test_split_kv_fused_combine_under_contention(gpu, attn_fused_all):
    """Decode batch with long contexts forced into 6 KV partitions: the in-launch
    last-ticket combine must give the same bits every launch and leave every
    semaphore re-armed (zero) for the next one."""
    from test_kernels_gpu import make_meta

    torch.manual_seed(3)
    np.random.seed(3)
    Hq, Hkv, NB = 32, 8, 1200
    q_lens = [1] * 12
    ctx_lens = [1500, 33, 900, 1400, 17, 1024, 1530, 640, 1, 1200, 777, 1499]
    kc = torch.randn(NB, Hkv, 16, 128, device=gpu, dtype=bf)
    vc = torch.randn(NB, Hkv, 16, 128, device=gpu, dtype=bf)
    m, T = make_meta(gpu, q_lens, ctx_lens, Hkv, Hq // Hkv, NB, part_tokens=256, nparts=6)
    m.part_sem = torch.zeros(m.tile_seq.numel() * Hkv, dtype=torch.int32, device=gpu)
    q = torch.randn(T, Hq, 128, device=gpu, dtype=bf)
    out = torch.empty_like(q)

    def launch():
        ops.paged_attention(q, kc, vc, m, out=out)
        return out

    y0, bad = _under_contention(gpu, launch, reps=40)
    assert not bad, f"fused split-KV combine changed on launches {bad}"
    assert int(m.part_sem.abs().sum()) == 0, "semaphores not re-armed"
    torch.testing.assert_close(y0.float(), ref.paged_attention(q, kc, vc, m).float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("M,N,K,epi", [(4088, 28672, 4096, 1), (4096, 4096, 14336, 0),
                                      (4088, 6144, 4096, 0), (2040, 28672, 4096, 1)])
def test_w4_gemm_under_contention(gpu, M, N, K, epi):
    """The four-wave GEMM's hand-counted LDS-DMA / ds_read waits (gemm_w4.hip): bit-identical
    results over many launches while a competing stream keeps the memory system busy (a
    read placed one wait too early shows up as rare wrong tiles under load), and the K-half
    tail tiles' sc1 partial hand-off (the last two shapes)."""
    torch.manual_seed(M + 1)
    ops._sk_reserve(torch.device(gpu))
    prev = torch.ops.mlop.gemm_big_variant(-1)
    torch.ops.mlop.gemm_big_variant(5)
    x = torch.randn(M, K, device=gpu, dtype=bf)
    w = (0.05 * torch.randn(N, K, device=gpu)).to(bf)
    ops.GEMM_BACKEND = "mlop"
    try:
        y0, bad = _under_contention(gpu, lambda: ops.gemm(x, w, epi=epi))
    finally:
        ops.GEMM_BACKEND = ops.GEMM_BACKEND_DEFAULT
        torch.ops.mlop.gemm_big_variant(prev)
    assert not bad, f"four-wave GEMM result changed on launches {bad}"
    exp = x.float() @ w.float().t()
    if epi:
        exp = ref.silu_mul(ops.deinterleave_cols(exp.to(bf)))
    tol = 3e-2 * exp.abs().max().item() / 10 + 1e-2
    torch.testing.assert_close(y0.float(), exp.float(), atol=tol, rtol=2e-2)
