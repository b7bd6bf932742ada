"""Building blocks shared by the model families: GEMM entry point, RoPE tables,
random on-device weight init (G4: no host-side materialisation of 16-141 GB).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .. import ops


def linear(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """y = x @ w^T with w stored [N, K] (row-major out-features).

    Routed through ``ops.gemm`` which picks the hand-written MFMA kernel for
    the shapes it covers and hipBLASLt for the rest (plain library GEMM)."""
    return ops.gemm(x, w, out=out) if hasattr(ops, "gemm") else F.linear(x, w, out=out)


def rope_inv_freq(head_dim: int, theta: float, scaling: dict | None = None) -> torch.Tensor:
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling.get("factor", 8.0)
        lo, hi = scaling.get("low_freq_factor", 1.0), scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        lo_wl, hi_wl = old / lo, old / hi
        wl = 2 * math.pi / inv
        smooth = (old / wl - lo) / (hi - lo)
        scaled = torch.where(wl > lo_wl, inv / factor, inv)
        mid = (wl <= lo_wl) & (wl >= hi_wl)
        inv = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
    return inv


def rope_table(head_dim: int, max_pos: int, theta: float, scaling: dict | None = None,
               device=None) -> torch.Tensor:
    """[max_pos, head_dim] fp32: cos in [:, :D/2], sin in [:, D/2:] (host-precomputed)."""
    inv = rope_inv_freq(head_dim, theta, scaling)
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return torch.cat([f.cos(), f.sin()], dim=-1).float().to(device)


def init_weight(shape, device, dtype=torch.bfloat16, std: float = 0.02, gen: torch.Generator | None = None):
    w = torch.empty(*shape, device=device, dtype=dtype)
    w.normal_(0.0, std, generator=gen)
    return w


def init_norm(n, device, dtype=torch.bfloat16):
    return torch.ones(n, device=device, dtype=dtype)
