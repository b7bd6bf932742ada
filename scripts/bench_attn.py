"""Decode paged-attention bandwidth at the headline's shape: B decode rows (Llama-3-8B GQA
32 q / 8 kv heads, D = 128, 16-token pages scattered over the pool), context lengths
uniform in [LO, HI] (the bench's steady state: 256-token prompts, 0..256 generated).
Reports us per call and the KV bytes read per second (K + V of every context token once)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlopamd import ops  # noqa: E402
from mlopamd.runtime.attn_meta import plan_partitions  # noqa: E402

ops.load()
dev = torch.device("cuda")
bf = torch.bfloat16
B = int(os.environ.get("B", "2048"))
LO, HI = (int(v) for v in os.environ.get("CTX", "256,512").split(","))
Hq, Hkv, D, BS = 32, 8, 128, 16
rng = np.random.default_rng(0)
ctx = rng.integers(LO, HI + 1, size=B).astype(np.int32)
pages = (ctx + BS - 1) // BS
NB = int(pages.sum()) + 16
MB = int(pages.max())
perm = rng.permutation(np.arange(1, NB))
bt = np.zeros((B, MB), np.int32)
p = 0
for i in range(B):
    bt[i, :pages[i]] = perm[p:p + pages[i]]
    p += pages[i]


class Meta:
    pass


m = Meta()
d = lambda a: torch.tensor(np.asarray(a), dtype=torch.int32, device=dev)  # noqa: E731
m.block_tables, m.ctx_len = d(bt), d(ctx)
m.q_start, m.q_len = d(np.arange(B)), d(np.ones(B))
m.tile_seq, m.tile_q0 = d(np.arange(B)), d(np.zeros(B))
m.ptile_seq = m.ptile_q0 = d(np.zeros(0))
m.part_tokens, m.nparts = plan_partitions(B, Hkv, int(ctx.max()))
if os.environ.get("PART"):  # forced partition length (tokens, multiple of 32)
    m.part_tokens = int(os.environ["PART"])
    m.nparts = (int(ctx.max()) + m.part_tokens - 1) // m.part_tokens
if m.nparts > 1:
    m.part_sem = torch.zeros(B * Hkv, dtype=torch.int32, device=dev)  # in-launch combine counters
m.part_o = torch.empty(B * Hkv * m.nparts * 16 * D, device=dev)
m.part_ml = torch.empty(B * Hkv * m.nparts * 16 * 2, device=dev)
kc = torch.randn(NB, Hkv, BS, D, device=dev, dtype=bf)
vc = torch.randn(NB, Hkv, BS, D, device=dev, dtype=bf)
q = torch.randn(B, Hq, D, device=dev, dtype=bf)
out = torch.empty_like(q)
for _ in range(3):
    ops.paged_attention(q, kc, vc, m, out=out)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
best = float("inf")
for _ in range(5):
    s.record()
    for _ in range(20):
        ops.paged_attention(q, kc, vc, m, out=out)
    e.record()
    e.synchronize()
    best = min(best, s.elapsed_time(e) / 20 * 1e3)
kv_bytes = int(ctx.sum()) * Hkv * D * 2 * 2
print(json.dumps(dict(B=B, ctx=[LO, HI], nparts=m.nparts, us=round(best, 1),
                      kv_gb=round(kv_bytes / 1e9, 3), tbps=round(kv_bytes / best / 1e6, 2))), flush=True)
