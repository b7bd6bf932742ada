"""A/B of the V page layout in the attention kernels: dim-major [NB, Hkv, 128, 16] (current)
vs token-major [NB, Hkv, 16, 128] staged through LDS and read with ds_read_b64_tr_b16
(MLOP_VT=1).  Same K / V values in both layouts: the outputs must be bit-identical; times are
interleaved per case.  Decode: B sequences x 1 token at context ~L (Llama-3-8B heads);
flash prefill: S prompts of L tokens in one chunk."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from mlopamd import ops  # noqa: E402
from test_kernels_gpu import make_meta  # noqa: E402

ops.load()
dev = torch.device("cuda")
bf = torch.bfloat16
Hq, Hkv, D, BS = 32, 8, 128, 16


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


def ab(run, vc_dm, label, extra):
    NB = vc_dm.shape[0]
    vc_tm = vc_dm.transpose(2, 3).contiguous().view(NB, Hkv, D, BS)  # token-major bytes, checked shape
    os.environ["MLOP_VT"] = "0"
    o0 = run(vc_dm).clone()
    os.environ["MLOP_VT"] = "1"
    o1 = run(vc_tm).clone()
    same = torch.equal(o0, o1)
    t = {"dm": [], "tm": []}
    for _ in range(3):
        os.environ["MLOP_VT"] = "0"
        t["dm"].append(timeit(lambda: run(vc_dm)))
        os.environ["MLOP_VT"] = "1"
        t["tm"].append(timeit(lambda: run(vc_tm)))
    os.environ["MLOP_VT"] = "0"
    r = dict(case=label, bit_identical=same, max_abs_diff=float((o0.float() - o1.float()).abs().max()),
             dm_us=round(min(t["dm"]), 1), tm_us=round(min(t["tm"]), 1))
    r.update(extra)
    print(json.dumps(r), flush=True)


for B, L in [(int(b), int(l)) for b, l in (c.split("x") for c in
             os.environ.get("CASES", "2048x384,1024x384,256x1024,64x4096,8x8192,1x8192").split(","))]:
    np.random.seed(0)
    ctx = np.random.randint(max(16, L // 2), L * 3 // 2 + 1, size=B).tolist()
    NB = sum((c + 15) // 16 for c in ctx) + 8
    kc = torch.randn(NB, Hkv, BS, D, device=dev, dtype=bf)
    vc = torch.randn(NB, Hkv, D, BS, device=dev, dtype=bf)
    m, T = make_meta(dev, [1] * B, ctx, Hkv, Hq // Hkv, NB)
    q = torch.randn(T, Hq, D, device=dev, dtype=bf)
    byts = sum(ctx) * Hkv * D * 2 * 2
    ab(lambda v: ops.paged_attention(q, kc, v, m), vc, f"decode {B}x{L}",
       dict(nparts=m.nparts, kv_gb=round(byts / 1e9, 3)))

# flash prefill
for S, L in [(int(a), int(b)) for a, b in (c.split("x") for c in os.environ.get("FCASES", "4x2048,1x8192").split(","))]:
    G = Hq // Hkv
    pqt = 128 // G
    rng = np.random.default_rng(0)
    pages = (L + BS - 1) // BS
    NB = S * pages + 16
    bt = rng.permutation(np.arange(1, NB))[:S * pages].reshape(S, pages).astype(np.int32)
    pts, ptq = [], []
    for s in range(S):
        n = (L + pqt - 1) // pqt
        pts += [s] * n
        ptq += list(range((n - 1) * pqt, -1, -pqt))

    class Meta:
        pass

    m = Meta()
    d = lambda a: torch.tensor(np.asarray(a), dtype=torch.int32, device=dev)  # noqa: E731
    m.block_tables, m.ctx_len = d(bt), d(np.full(S, L))
    m.q_start, m.q_len = d(np.arange(S) * L), d(np.full(S, L))
    m.tile_seq = m.tile_q0 = d(np.zeros(0))
    m.ptile_seq, m.ptile_q0 = d(pts), d(ptq)
    m.part_tokens, m.nparts = L, 1
    m.part_o = m.part_ml = torch.empty(1, device=dev)
    kc = torch.randn(NB, Hkv, BS, D, device=dev, dtype=bf)
    vc = torch.randn(NB, Hkv, D, BS, device=dev, dtype=bf)
    q = torch.randn(S * L, Hq, D, device=dev, dtype=bf)
    out = torch.empty_like(q)
    flops = 4 * S * (L * (L + 1) // 2) * D * Hq
    ab(lambda v: ops.paged_attention(q, kc, v, m, out=out), vc, f"flash {S}x{L}", dict(gflop=round(flops / 1e9, 1)))
