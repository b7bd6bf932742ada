"""Dense (no KV cache, no paging) fp32 re-computation of a model's logits.

Independent oracle for the engine: it shares only the weights with the
serving path (no kernels, no metadata, no paging), so paging / chunking /
graph bugs show up as logit mismatches.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..ops import deinterleave_rows
from ..ops import reference as ref


def _mlp(model, i, x):
    L = model.layers[i]
    if model.cfg.is_moe:
        logits = F.linear(x, L["router"].float())
        w, idx = torch.topk(torch.softmax(logits, -1), model.cfg.top_k, dim=-1)
        w = w / w.sum(-1, keepdim=True)
        out = torch.zeros_like(x)
        for e in range(model.cfg.num_experts):
            rows, k = (idx == e).nonzero(as_tuple=True)
            if rows.numel() == 0:
                continue
            gu = F.linear(x[rows], deinterleave_rows(L["w13"][e]).float())
            h = F.linear(ref.silu_mul(gu.to(model.dtype)).float(), L["w2"][e].float())
            out.index_add_(0, rows, h * w[rows, k, None])
        return out
    gu = F.linear(x, deinterleave_rows(L["gate_up"]).float()).to(model.dtype)
    return F.linear(ref.silu_mul(gu).float(), L["down"].float())


@torch.no_grad()
def dense_logits(model, tokens) -> torch.Tensor:
    """[T, V] fp32 logits of a single sequence (TP=1 models only)."""
    cfg = model.cfg
    dev = model.embed.device
    T = len(tokens)
    ids = torch.tensor(tokens, device=dev)
    res = model.embed[ids].float()
    x = ref.rmsnorm(res, model.layers[0]["in_norm"].float(), cfg.rms_eps)
    cs = model.cos_sin[torch.arange(T, device=dev)]
    D, half = cfg.head_dim, cfg.head_dim // 2
    G = model.n_q // model.n_kv
    mask = torch.triu(torch.ones(T, T, dtype=torch.bool, device=dev), 1)
    for i, L in enumerate(model.layers):
        qkv = F.linear(x, L["qkv"].float())
        q = qkv[:, : model.n_q * D].view(T, model.n_q, D)
        k = qkv[:, model.n_q * D:(model.n_q + model.n_kv) * D].view(T, model.n_kv, D)
        v = qkv[:, (model.n_q + model.n_kv) * D:].view(T, model.n_kv, D)
        q = ref.rotate(q, cs[:, None, :half], cs[:, None, half:])
        k = ref.rotate(k, cs[:, None, :half], cs[:, None, half:]).repeat_interleave(G, 1)
        v = v.repeat_interleave(G, 1)
        s = torch.einsum("qhd,khd->hqk", q, k) / D ** 0.5
        s = s.masked_fill(mask[None], float("-inf"))
        a = torch.einsum("hqk,khd->qhd", s.softmax(-1), v).reshape(T, -1)
        res = res + F.linear(a, L["o"].float())
        x = ref.rmsnorm(res, L["post_norm"].float(), cfg.rms_eps)
        res = res + _mlp(model, i, x)
        nxt = model.layers[i + 1]["in_norm"] if i + 1 < len(model.layers) else model.final_norm
        x = ref.rmsnorm(res, nxt.float(), cfg.rms_eps)
    return F.linear(x, model.lm_head.float())
