"""Mixture-of-experts dispatch / compute / combine (K11-K14, CL4).

Two placements of the experts of one MoE layer over an EP group:

* ``allreduce`` — tokens are replicated over the group (TP attention): every
  rank runs its E/ep local experts on the rows routed to them and the partial
  outputs are summed by the layer's TP all-reduce (no all-to-all).
* ``alltoall`` — tokens are sharded over the group (DP attention + EP MoE):
  routed rows go to the rank owning their expert with an all-to-all (dispatch),
  are computed there with the grouped GEMM, and come back with a second
  all-to-all (combine), then the top-k weights are applied at the source.

On GPU the routing, permutation, grouped GEMM and combine are HIP kernels
(``ops.moe_*``); CPU tensors run the reference path.
"""
from __future__ import annotations

import torch

from .. import ops
from ..models.layers import linear


def route(x: torch.Tensor, router_w: torch.Tensor, top_k: int):
    """softmax(x @ Wr^T) -> top-k -> renormalised weights (Mixtral). fp32 [T,k], int32 [T,k]."""
    logits = linear(x, router_w)
    return ops.moe_route(logits, top_k)


def local_experts(x, topw, topi, w13, w2, e0: int, n_local: int, dispatched=None, combine: bool = True):
    """Sum over the top-k slots whose expert is in [e0, e0+n_local) of w * expert(x).

    permute (K12) -> grouped gate_up GEMM with fused SiLU-mul (K13, w13 rows
    gate/up-interleaved) -> grouped down GEMM (K13) -> weighted gather (K14).
    ``dispatched``: (xp, offsets, inv) from ops.moe_dispatch_small; ``combine=False``
    returns (y, inv) so the caller can fuse the weighted gather into its next kernel."""
    T, k = topi.shape
    if dispatched is None:
        xp, offsets, src, inv = ops.moe_permute(x, topi, e0, n_local)
    else:
        xp, offsets, inv = dispatched
    avg = max(1, (T * k) // max(1, n_local))
    a = ops.grouped_gemm(xp, w13, offsets, epi=ops.EPI_SILU_MUL, avg_rows=avg)
    y = ops.grouped_gemm(a, w2, offsets, avg_rows=avg)
    return ops.moe_combine(y, inv, topw) if combine else (y, inv)


def moe_forward_add_norm(x, router_w, w13, w2, top_k: int, e0: int, n_local: int, residual, norm_w, eps: float,
                         pre=None):
    """Single-rank MoE block followed by the decoder's residual add + RMSNorm.  At decode
    sizes the router GEMV, routing, sort and gather are ONE launch (moe_dispatch_small) and
    the weighted combine rides in the add + RMSNorm launch: 6 MoE glue launches -> 2.
    ``pre=(o, pre_norm_w)``: x is not formed yet; the block's own input add + RMSNorm
    (residual += o, x = rmsnorm(residual)) becomes the dispatch launch's prologue."""
    if pre is not None:
        o, pre_w = pre
        d = ops.moe_dispatch_small(o, router_w, top_k, e0, n_local, pro=(o, residual, pre_w, eps))
        if d is None:
            x = ops.add_rmsnorm(o, residual, pre_w, eps)
    else:
        d = ops.moe_dispatch_small(x, router_w, top_k, e0, n_local)
    if d is None:
        topw, topi = route(x, router_w, top_k)
        y, inv = local_experts(x, topw, topi, w13, w2, e0, n_local, combine=False)
    else:
        topw, topi, xp, offsets, _src, inv = d
        y, inv = local_experts(x, topw, topi, w13, w2, e0, n_local, dispatched=(xp, offsets, inv), combine=False)
    return ops.moe_combine_add_rmsnorm(y, inv, topw, residual, norm_w, eps)


def moe_forward(x, router_w, w13, w2, top_k: int, ep, e0: int, n_local: int, mode: str = "allreduce"):
    topw, topi = route(x, router_w, top_k)
    if ep.size == 1 or mode == "allreduce":
        return local_experts(x, topw, topi, w13, w2, e0, n_local)
    return _alltoall(x, topw, topi, w13, w2, top_k, ep, n_local)


def _alltoall(x, topw, topi, w13, w2, top_k, ep, n_local):
    """Expert-parallel MoE with RCCL all-to-all dispatch and combine."""
    import torch.distributed as dist

    T, H = x.shape
    P = ep.size
    flat_e = topi.reshape(-1).long()                      # [T*k]
    dest = flat_e // n_local                              # owning rank of each routed row
    order = torch.argsort(dest, stable=True)
    send_rows = x.index_select(0, order // top_k)         # [T*k, H] grouped by destination
    send_e = (flat_e[order] % n_local).to(torch.int32)    # local expert id at the destination
    send_counts = torch.bincount(dest, minlength=P)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=ep.handle)
    sc, rc = send_counts.tolist(), recv_counts.tolist()
    n_recv = sum(rc)
    recv_rows = torch.empty(n_recv, H, dtype=x.dtype, device=x.device)
    recv_e = torch.empty(n_recv, dtype=torch.int32, device=x.device)
    dist.all_to_all_single(recv_rows, send_rows, rc, sc, group=ep.handle)
    dist.all_to_all_single(recv_e, send_e, rc, sc, group=ep.handle)
    # compute the received rows with the local experts (weight 1: scaled at the source)
    ones = torch.ones(n_recv, 1, dtype=torch.float32, device=x.device)
    y = local_experts(recv_rows, ones, recv_e.view(-1, 1), w13, w2, 0, n_local)
    back = torch.empty(T * top_k, H, dtype=x.dtype, device=x.device)
    dist.all_to_all_single(back, y, sc, rc, group=ep.handle)
    # un-permute to [T, k, H] and apply the routing weights
    slot_rows = torch.empty_like(back)
    slot_rows[order] = back
    out = (slot_rows.view(T, top_k, H).float() * topw[..., None]).sum(1)
    return out.to(x.dtype)
