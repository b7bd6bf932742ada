"""Plain PyTorch (fp32 math) definitions of every HIP op.

They are the numerics oracle of the GPU tests (``tests/test_kernels_gpu.py``)
and the execution path for CPU tensors, so the scheduler / engine / TP logic is
unit-testable in a GPU-less container.  Layouts match the kernels exactly:
``k_cache[NB, Hkv, BS, D]`` and ``v_cache[NB, Hkv, BS, D]`` (both token-major).
"""
from __future__ import annotations

import math

import torch


def rmsnorm(x, w, eps):
    xf = x.float()
    inv = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (w.float() * (xf * inv).to(x.dtype).float()).to(x.dtype)


def add_rmsnorm(x, residual, w, eps):
    r = (x.float() + residual.float()).to(x.dtype)
    return rmsnorm(r, w, eps), r


def silu_mul(x):
    I = x.shape[-1] // 2
    g, u = x[..., :I].float(), x[..., I:].float()
    return (torch.nn.functional.silu(g).to(x.dtype).float() * u).to(x.dtype)


def embedding(ids, table, vocab_start=0):
    ids = ids.reshape(-1).long()
    local = ids - vocab_start
    ok = (local >= 0) & (local < table.shape[0])
    out = table[local.clamp(0, table.shape[0] - 1)].clone()
    out[~ok] = 0
    return out


def rotate(x, cos, sin):
    half = x.shape[-1] // 2
    x1, x2 = x[..., :half], x[..., half:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1)


def rope_cache(qkv, positions, cos_sin, slots, k_cache, v_cache, n_q_heads):
    """Rotate q/k, scatter k/v into the paged cache, return q [T, Hq, D]."""
    T = qkv.shape[0]
    Hkv, BS, D = k_cache.shape[1], k_cache.shape[2], k_cache.shape[3]
    half = D // 2
    x = qkv[:, : (n_q_heads + 2 * Hkv) * D].float().view(T, n_q_heads + 2 * Hkv, D)
    cs = cos_sin[positions.long()].float()  # [T, D]
    cos, sin = cs[:, None, :half], cs[:, None, half:]
    q = rotate(x[:, :n_q_heads], cos, sin).to(qkv.dtype)
    k = rotate(x[:, n_q_heads:n_q_heads + Hkv], cos, sin).to(qkv.dtype)
    v = x[:, n_q_heads + Hkv:].to(qkv.dtype)
    for t in range(T):
        s = int(slots[t])
        if s < 0:
            continue
        b, o = divmod(s, BS)
        k_cache[b, :, o, :] = k[t]
        v_cache[b, :, o, :] = v[t]
    return q


def gather_kv(k_cache, v_cache, block_table, n):
    """Contiguous K, V [n, Hkv, D] of one sequence from its pages."""
    BS = k_cache.shape[2]
    pages = [int(p) for p in block_table[: (n + BS - 1) // BS]]
    if not pages:
        Hkv, D = k_cache.shape[1], k_cache.shape[3]
        z = torch.zeros(0, Hkv, D, dtype=k_cache.dtype, device=k_cache.device)
        return z, z
    k = torch.cat([k_cache[p].permute(1, 0, 2) for p in pages], 0)[:n]          # [n, Hkv, D]
    v = torch.cat([v_cache[p].permute(1, 0, 2) for p in pages], 0)[:n]          # [n, Hkv, D]
    return k, v


def paged_attention(q, k_cache, v_cache, meta):
    """Causal GQA attention of every query token of ``meta`` over its paged context."""
    out = torch.zeros_like(q)
    Hq, D = q.shape[1], q.shape[2]
    Hkv = k_cache.shape[1]
    G = Hq // Hkv
    scale = 1.0 / math.sqrt(D)
    qs, ql, cl = (meta.q_start.cpu().tolist(), meta.q_len.cpu().tolist(), meta.ctx_len.cpu().tolist())
    bt = meta.block_tables.cpu()
    # only rows referenced by this launch's tiles are live (other rows hold stale values)
    live = set(meta.tile_seq.cpu().tolist())
    if getattr(meta, "ptile_seq", None) is not None:
        live |= set(meta.ptile_seq.cpu().tolist())
    for s in sorted(live):
        if ql[s] == 0 or cl[s] == 0:
            continue
        k, v = gather_kv(k_cache, v_cache, bt[s], cl[s])
        k = k.float().repeat_interleave(G, dim=1)  # [n, Hq, D]
        v = v.float().repeat_interleave(G, dim=1)
        qq = q[qs[s]:qs[s] + ql[s]].float()      # [ql, Hq, D]
        scores = torch.einsum("qhd,khd->hqk", qq, k) * scale
        pos = torch.arange(cl[s] - ql[s], cl[s], device=q.device)[:, None]
        keys = torch.arange(cl[s], device=q.device)[None, :]
        scores = scores.masked_fill((keys > pos)[None], float("-inf"))
        p = torch.softmax(scores, dim=-1)
        out[qs[s]:qs[s] + ql[s]] = torch.einsum("hqk,khd->qhd", p, v).to(q.dtype)
    return out


# ------------------------------------------------------------------ MoE --

def moe_route(logits, top_k):
    p = torch.softmax(logits.float(), dim=-1)
    w, idx = torch.topk(p, top_k, dim=-1)
    w = w / w.sum(-1, keepdim=True)
    return w, idx.to(torch.int32)


def moe_permute(x, topi, e0, n_local):
    """Rows routed to local experts, grouped by expert (stable in slot order), padded to T*k rows.
    Returns (xp [T*k, H], offsets int32 [n_local+1], src int32 [T*k], inv int32 [T*k])."""
    T, k = topi.shape
    flat = topi.reshape(-1).long() - e0
    ok = (flat >= 0) & (flat < n_local)
    slots = torch.nonzero(ok, as_tuple=True)[0]
    e = flat[slots]
    order = torch.argsort(e, stable=True)
    slots, e = slots[order], e[order]
    n = slots.numel()
    counts = torch.bincount(e, minlength=n_local)
    offsets = torch.zeros(n_local + 1, dtype=torch.int32, device=x.device)
    offsets[1:] = torch.cumsum(counts, 0).to(torch.int32)
    xp = torch.zeros(T * k, x.shape[1], dtype=x.dtype, device=x.device)
    xp[:n] = x[slots // k]
    src = torch.full((T * k,), -1, dtype=torch.int32, device=x.device)
    src[:n] = slots.to(torch.int32)
    inv = torch.full((T * k,), -1, dtype=torch.int32, device=x.device)
    inv[slots] = torch.arange(n, dtype=torch.int32, device=x.device)
    return xp, offsets, src, inv


def grouped_gemm(xp, w, offsets):
    """Per group e: rows [off[e], off[e+1]) of xp times w[e]^T (w: [E, N, K]); other rows 0."""
    out = torch.zeros(xp.shape[0], w.shape[1], dtype=xp.dtype, device=xp.device)
    off = offsets.tolist()
    for e in range(w.shape[0]):
        a, b = off[e], off[e + 1]
        if b > a:
            out[a:b] = (xp[a:b].float() @ w[e].float().t()).to(xp.dtype)
    return out


def moe_combine(y, inv, topw):
    T, k = topw.shape
    out = torch.zeros(T, y.shape[1], dtype=torch.float32, device=y.device)
    inv = inv.long().view(T, k)
    for j in range(k):
        ok = inv[:, j] >= 0
        if ok.any():
            out[ok] += topw[ok, j, None].float() * y[inv[ok, j]].float()
    return out.to(y.dtype)
