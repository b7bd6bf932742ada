"""K7 flash-prefill microbench: S fresh prompts of L tokens each in ONE chunk (causal),
Llama-3-8B GQA (32 q / 8 kv heads, D = 128), K/V already in scattered 16-token pages.
Reports us per call and causal attention TFLOP/s (QK^T + PV, 4 * sum(pos+1) * D * Hq)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlopamd import ops  # noqa: E402

ops.load()
dev = torch.device("cuda")
bf = torch.bfloat16
S = int(os.environ.get("S", "4"))
L = int(os.environ.get("L", "2048"))
ITERS = int(os.environ.get("ITERS", "20"))
Hq, Hkv, D, BS = 32, 8, 128, 16
G = Hq // Hkv
pqt = 128 // G
rng = np.random.default_rng(0)
pages = (L + BS - 1) // BS
NB = S * pages + 16
perm = rng.permutation(np.arange(1, NB))
bt = perm[:S * pages].reshape(S, pages).astype(np.int32)
q_start = np.arange(S, dtype=np.int32) * L
pts, ptq = [], []
for s in range(S):  # latest tiles first (the longest causal ranges dispatch first)
    n = (L + pqt - 1) // pqt
    pts += [s] * n
    ptq += list(range((n - 1) * pqt, -1, -pqt))
if os.environ.get("ORDER", "lpt") == "lpt":  # attn_meta.order_flash_tiles (the engine: prompts >= 1024)
    from mlopamd.runtime.attn_meta import order_flash_tiles

    pts, ptq = np.asarray(pts, dtype=np.int32), np.asarray(ptq, dtype=np.int32)
    order_flash_tiles(pts, ptq, (ptq + pqt).astype(np.int32))


class Meta:
    pass


m = Meta()
d = lambda a: torch.tensor(np.asarray(a), dtype=torch.int32, device=dev)  # noqa: E731
m.block_tables, m.ctx_len = d(bt), d(np.full(S, L))
m.q_start, m.q_len = d(q_start), d(np.full(S, L))
m.tile_seq = m.tile_q0 = d(np.zeros(0))
m.ptile_seq, m.ptile_q0 = d(pts), d(ptq)
m.part_tokens, m.nparts = L, 1
m.part_o = m.part_ml = torch.empty(1, device=dev)
kc = torch.randn(NB, Hkv, BS, D, device=dev, dtype=bf)
vc = torch.randn(NB, Hkv, BS, D, device=dev, dtype=bf)
q = torch.randn(S * L, Hq, D, device=dev, dtype=bf)
out = torch.empty_like(q)
flops = 4 * S * (L * (L + 1) // 2) * D * Hq
# PERSIST: flash_persist values to interleave (0 = one workgroup per item; n = the persistent
# grid with n workgroups per CU; an "s" suffix runs it as the cross-tile stream, flash_stream 1),
# e.g. "0,3,2s"
for pvs in os.environ.get("PERSIST", str(torch.ops.mlop.flash_persist(-1))).split(","):
    pv = int(pvs.rstrip("s"))
    torch.ops.mlop.flash_persist(pv)
    torch.ops.mlop.flash_stream(1 if pvs.endswith("s") else 0)
    for _ in range(3):
        ops.paged_attention(q, kc, vc, m, out=out)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    best = float("inf")
    for _ in range(3):
        ev[0].record()
        for _ in range(ITERS):
            ops.paged_attention(q, kc, vc, m, out=out)
        ev[1].record()
        ev[1].synchronize()
        best = min(best, ev[0].elapsed_time(ev[1]) / ITERS * 1e3)
    line = dict(S=S, L=L, order=os.environ.get("ORDER", "lpt"), persist=pvs, tiles=len(pts), us=round(best, 1),
                tflops=round(flops / best / 1e6, 1))
    if os.environ.get("CHECK"):
        from mlopamd.ops import reference as ref

        out.zero_()
        ops.paged_attention(q, kc, vc, m, out=out)
        exp = ref.paged_attention(q, kc, vc, m)
        line["max_abs_err"] = (out.float() - exp.float()).abs().max().item()
    print(json.dumps(line), flush=True)
