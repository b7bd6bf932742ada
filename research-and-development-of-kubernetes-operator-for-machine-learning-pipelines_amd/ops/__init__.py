"""Hand-written gfx950 HIP kernels, exposed as ``torch.ops.mlop.*``.

``load()`` loads the in-tree ``_C.so`` (built by ``mlopamd.ops.build``).  On a
GPU process the extension is REQUIRED: every public function here raises if it
is missing instead of silently running a PyTorch fallback.  CPU tensors (unit
tests of the scheduler / engine logic in a GPU-less container) are routed to
``mlopamd.ops.reference`` — the plain fp32 PyTorch definitions that the GPU
numerics tests also use as their oracle.
"""
from __future__ import annotations

import math
import os
from pathlib import Path

import torch

from . import reference as ref

_LIB = Path(__file__).resolve().parent / "_C.so"
_loaded = False


def load(build_if_missing: bool = True) -> bool:
    """Load the extension; build it first if it is missing and hipcc exists."""
    global _loaded
    if _loaded:
        return True
    if not _LIB.exists() and build_if_missing:
        from .build import build

        build()
    torch.ops.load_library(str(_LIB))
    _loaded = True
    return True


def available() -> bool:
    try:
        return load(build_if_missing=False)
    except Exception:  # noqa: BLE001
        return False


def _need_gpu():
    if not _loaded:
        load()


def library_path() -> str:
    return str(_LIB)


# ---------------------------------------------------------------- wrappers --

def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, out: torch.Tensor | None = None):
    if not x.is_cuda:
        return ref.rmsnorm(x, w, eps)
    _need_gpu()
    out = torch.empty_like(x) if out is None else out
    torch.ops.mlop.rmsnorm(out, x, w, eps)
    return out


def add_rmsnorm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float,
                out: torch.Tensor | None = None):
    """residual <- residual + x (bf16); returns rmsnorm(residual) * w."""
    if not x.is_cuda:
        y, r = ref.add_rmsnorm(x, residual, w, eps)
        residual.copy_(r)
        return y
    _need_gpu()
    out = torch.empty_like(x) if out is None else out
    torch.ops.mlop.add_rmsnorm(out, residual, x, w, eps)
    return out


def rope_cache(qkv, positions, cos_sin, slots, k_cache, v_cache, n_q_heads: int,
               q_out: torch.Tensor | None = None):
    T = qkv.shape[0]
    D = k_cache.shape[3]
    if not qkv.is_cuda:
        q = ref.rope_cache(qkv, positions, cos_sin, slots, k_cache, v_cache, n_q_heads)
        if q_out is not None:
            q_out.copy_(q)
            return q_out
        return q
    _need_gpu()
    q_out = torch.empty(T, n_q_heads, D, dtype=qkv.dtype, device=qkv.device) if q_out is None else q_out
    torch.ops.mlop.rope_cache(q_out, k_cache, v_cache, qkv, positions, cos_sin, slots)
    return q_out


def silu_mul(x: torch.Tensor, out: torch.Tensor | None = None):
    if not x.is_cuda:
        return ref.silu_mul(x)
    _need_gpu()
    I = x.shape[-1] // 2
    out = torch.empty(*x.shape[:-1], I, dtype=x.dtype, device=x.device) if out is None else out
    torch.ops.mlop.silu_mul(out, x)
    return out


def embedding(ids: torch.Tensor, table: torch.Tensor, vocab_start: int = 0,
              out: torch.Tensor | None = None):
    if not ids.is_cuda:
        return ref.embedding(ids, table, vocab_start)
    _need_gpu()
    out = torch.empty(ids.numel(), table.shape[1], dtype=table.dtype, device=table.device) if out is None else out
    torch.ops.mlop.embedding(out, table, ids, vocab_start)
    return out


def paged_attention(q, k_cache, v_cache, meta, out: torch.Tensor | None = None):
    """Ragged paged attention; ``meta`` is a ``mlopamd.runtime.attn_meta.AttnMeta``."""
    if not q.is_cuda:
        return ref.paged_attention(q, k_cache, v_cache, meta)
    _need_gpu()
    out = torch.empty_like(q) if out is None else out
    scale = 1.0 / math.sqrt(q.shape[-1])
    torch.ops.mlop.paged_attention(out, meta.part_o, meta.part_ml, q, k_cache, v_cache,
                                   meta.block_tables, meta.tile_seq, meta.tile_q0, meta.q_start,
                                   meta.q_len, meta.ctx_len, scale, meta.part_tokens, meta.nparts)
    return out


def argmax(logits: torch.Tensor) -> torch.Tensor:
    if not logits.is_cuda:
        return logits.argmax(-1)
    _need_gpu()
    out = torch.empty(logits.shape[0], dtype=torch.int64, device=logits.device)
    torch.ops.mlop.argmax(out, logits)
    return out


def sample(logits, temps, top_ks, top_ps, uniform) -> torch.Tensor:
    if not logits.is_cuda:
        from ..runtime.sampler import sample_reference

        return sample_reference(logits, temps, top_ks, top_ps, uniform)
    _need_gpu()
    out = torch.empty(logits.shape[0], dtype=torch.int64, device=logits.device)
    torch.ops.mlop.sample(out, logits, temps, top_ks, top_ps, uniform)
    return out


__all__ = ["argmax", "sample", "load","available", "library_path", "rmsnorm", "add_rmsnorm", "rope_cache",
           "silu_mul", "embedding", "paged_attention", "ref"]


# ------------------------------------------------------------------ MoE --

def _has(name: str) -> bool:
    _need_gpu()
    return hasattr(torch.ops.mlop, name)


def moe_route(logits: torch.Tensor, top_k: int):
    if not logits.is_cuda or not _has("moe_route"):
        return ref.moe_route(logits, top_k)
    T, E = logits.shape
    w = torch.empty(T, top_k, dtype=torch.float32, device=logits.device)
    idx = torch.empty(T, top_k, dtype=torch.int32, device=logits.device)
    torch.ops.mlop.moe_route(w, idx, logits.contiguous())
    return w, idx


def moe_permute(x, topi, e0: int, n_local: int):
    if not x.is_cuda or not _has("moe_permute"):
        return ref.moe_permute(x, topi, e0, n_local)
    T, k = topi.shape
    xp = torch.empty(T * k, x.shape[1], dtype=x.dtype, device=x.device)
    offsets = torch.empty(n_local + 1, dtype=torch.int32, device=x.device)
    src = torch.empty(T * k, dtype=torch.int32, device=x.device)
    n = torch.ops.mlop.moe_permute(xp, offsets, src, x, topi, e0, n_local)
    return xp[:n], offsets, src[:n]


def grouped_gemm(xp, w, offsets):
    if not xp.is_cuda or not _has("grouped_gemm"):
        return ref.grouped_gemm(xp, w, offsets)
    out = torch.empty(xp.shape[0], w.shape[1], dtype=xp.dtype, device=xp.device)
    torch.ops.mlop.grouped_gemm(out, xp, w, offsets)
    return out


def moe_combine(y, src, topw, T: int):
    if not y.is_cuda or not _has("moe_combine"):
        return ref.moe_combine(y, src, topw, T)
    out = torch.empty(T, y.shape[1], dtype=y.dtype, device=y.device)
    torch.ops.mlop.moe_combine(out, y, src, topw)
    return out
