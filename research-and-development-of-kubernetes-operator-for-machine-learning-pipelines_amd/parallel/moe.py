"""Mixture-of-experts dispatch / compute / combine (K11-K14, CL4).

Two placements of the experts of one MoE layer over an EP group:

* ``allreduce`` — tokens are replicated over the group (TP attention): every
  rank runs its E/ep local experts on the rows routed to them and the partial
  outputs are summed by the layer's TP all-reduce (no all-to-all).
* ``alltoall`` — tokens are sharded over the group (DP attention + EP MoE):
  routed rows go to the rank owning their expert (dispatch), are computed there
  with the grouped GEMM, and come back (combine), then the top-k weights are
  applied at the source.  On GPU the exchange is device-side over IPC peer
  memory (``_ep_ipc``: exact, sync-free, graph-capturable); the padded RCCL /
  gloo ``all_to_all_single`` pair (``_alltoall``) is the CPU reference.

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


def local_experts(x, topw, topi, w13, w2, e0: int, n_local: int, dispatched=None, combine=True):
    """Sum over the top-k slots whose expert is in [e0, e0+n_local) of w * expert(x).

    permute (K12) -> grouped gate_up GEMM with fused SiLU-mul (K13, w13 rows
    gate/up-interleaved) -> grouped down GEMM (K13) -> weighted gather (K14).
    ``dispatched``: (xp, offsets, inv) from ops.moe_dispatch_small; ``combine=False``
    returns (y, inv) so the caller can fuse the weighted gather into its next kernel;
    ``combine=(residual, norm_w, eps)`` runs the down GEMM, the combine and the residual add +
    RMSNorm as one op (ops.moe_down_combine_add_rmsnorm) and returns the normed rows."""
    T, k = topi.shape
    arow = None
    if dispatched is None:
        xp, offsets, src, inv = ops.moe_permute(x, topi, e0, n_local)
    elif len(dispatched) == 4:  # moe_dispatch_mid: the token rows, read through arow (no gather)
        xp, offsets, inv, arow = dispatched
    else:
        xp, offsets, inv = dispatched
    avg = max(1, (T * k) // max(1, n_local))
    a = ops.grouped_gemm(xp, w13, offsets, epi=ops.EPI_SILU_MUL, avg_rows=avg, a_rows=arow)
    if isinstance(combine, tuple):
        residual, norm_w, eps = combine
        return ops.moe_down_combine_add_rmsnorm(a, w2, offsets, inv, topw, residual, norm_w, eps, avg)
    y = ops.grouped_gemm(a, w2, offsets, avg_rows=avg)
    return ops.moe_combine(y, inv, topw) if combine else (y, inv)


def moe_forward_add_norm(x, router_w, w13, w2, top_k: int, e0: int, n_local: int, residual, norm_w, eps: float,
                         pre=None):
    """Single-rank MoE block followed by the decoder's residual add + RMSNorm.  At decode
    sizes the router GEMV, routing, sort and gather are ONE launch (moe_dispatch_small; at
    16 < T <= 16384 moe_dispatch_mid, whose experts read x in place) and the weighted combine
    rides in the add + RMSNorm launch: 6 MoE glue launches -> 2.
    ``pre=(o, pre_norm_w)``: x is not formed yet; the block's own input add + RMSNorm
    (residual += o, x = rmsnorm(residual)) becomes the dispatch launch's prologue."""
    mid = None
    if pre is not None:
        o, pre_w = pre
        d = ops.moe_dispatch_small(o, router_w, top_k, e0, n_local, pro=(o, residual, pre_w, eps))
        if d is None:
            mid = ops.moe_dispatch_mid(o, router_w, top_k, e0, n_local, pro=(o, residual, pre_w, eps))
        if d is None and mid is None:
            x = ops.add_rmsnorm(o, residual, pre_w, eps)
    else:
        d = ops.moe_dispatch_small(x, router_w, top_k, e0, n_local)
        if d is None:
            mid = ops.moe_dispatch_mid(x, router_w, top_k, e0, n_local)
    if mid is not None:  # 16 < T <= 16384: one dispatch launch, the experts read x through arow
        topw, topi, xs, offsets, arow, inv = mid
        return local_experts(xs, topw, topi, w13, w2, e0, n_local, dispatched=(xs, offsets, inv, arow),
                             combine=(residual, norm_w, eps))
    if d is None:
        topw, topi = route(x, router_w, top_k)
        y, inv = local_experts(x, topw, topi, w13, w2, e0, n_local, combine=False)
    else:
        topw, topi, xp, offsets, _src, inv = d
        y, inv = local_experts(x, topw, topi, w13, w2, e0, n_local, dispatched=(xp, offsets, inv), combine=False)
    return ops.moe_combine_add_rmsnorm(y, inv, topw, residual, norm_w, eps)


def moe_forward(x, router_w, w13, w2, top_k: int, ep, e0: int, n_local: int, mode: str = "allreduce",
                cap_tokens: int | None = None):
    topw, topi = route(x, router_w, top_k)
    if ep.size == 1 or mode == "allreduce":
        return local_experts(x, topw, topi, w13, w2, e0, n_local)
    ex = getattr(ep, "ex", None)
    if x.is_cuda and ex is not None:
        return _ep_ipc(x, topw, topi, w13, w2, ex, cap_tokens)
    return _alltoall(x, topw, topi, w13, w2, top_k, ep, n_local, cap_tokens)


def _ep_ipc(x, topw, topi, w13, w2, ex, cap_tokens: int | None = None):
    """Expert-parallel MoE on GPU over IPC peer memory (parallel/ep_ipc.py, ep_exchange.hip):
    routed rows land in their owner's buffer already grouped by expert (exact counts, no
    padding rows on the fabric, no host sync), the owner runs its experts' grouped GEMM pair
    (K13) on them with device offsets, and the outputs go back to the source slots for the
    top-k weighted combine.  ``cap_tokens``: the group's agreed largest T this step (sizes the
    received-row buffer and the grouped GEMM grid; rows past the received count are never
    read)."""
    T = x.shape[0]
    xp, offsets = ex.dispatch(x, topi, cap_tokens or T)
    avg = max(1, (T * ex.k) // max(1, ex.n_local))
    a = ops.grouped_gemm(xp, w13, offsets, epi=ops.EPI_SILU_MUL, avg_rows=avg)
    y = ops.grouped_gemm(a, w2, offsets, avg_rows=avg)
    return ex.combine(y, topw, topi, T)


def _alltoall(x, topw, topi, w13, w2, top_k, ep, n_local, cap_tokens: int | None = None):
    """Expert-parallel MoE (DP attention: every rank holds different tokens) with all-to-all
    dispatch and combine and NO host synchronisation (graph-capturable, CL4):

      * this rank's routed rows are grouped by DESTINATION rank with the MoE permute kernel
        (K12, the owning rank standing in for the expert), then scattered into a fixed-capacity
        send buffer [P, C, H], C = cap_tokens * top_k (the worst case: every routed row of
        a rank goes to one peer), with each row's local expert id beside it (-1 = padding);
      * ONE equal-split all_to_all_single of rows (+ one of ids): no counts ever reach the
        host (RCCL over xGMI on GPU; the old path synced ``send_counts.tolist()``);
      * the received rows run through this rank's experts in ONE grouped GEMM pair (K13;
        padding rows carry expert -1 and are skipped by the permute);
      * the outputs go back with a second all-to-all into the same slots and the top-k
        weighted combine (K14) reads them in place.
    ``cap_tokens`` must be the same on every rank of the group (the engine agrees on the
    step's largest token count); default: this rank's T.  The exchange is exact (no token
    is dropped); its price is P x C rows per direction instead of the routed rows."""
    import torch.distributed as dist

    T, H = x.shape
    P, k = ep.size, top_k
    C = (T if cap_tokens is None else int(cap_tokens)) * k
    dev = x.device
    dest = torch.div(topi, n_local, rounding_mode="floor").to(torch.int32)  # owning rank per slot
    xp, offs, src, inv = ops.moe_permute(x, dest, 0, P)                    # rows sorted by dest
    n = T * k
    i = torch.arange(n, device=dev, dtype=torch.int64)
    d_sorted = torch.searchsorted(offs[1:].to(torch.int64), i, right=True)  # dest of sorted row i
    pos = d_sorted * C + (i - offs.to(torch.int64)[d_sorted])               # slot in the send buffer
    send = torch.zeros(P * C, H, dtype=x.dtype, device=dev)
    send.index_copy_(0, pos, xp[:n])
    e_loc = torch.full((P * C,), -1, dtype=torch.int32, device=dev)
    e_loc.index_copy_(0, pos, torch.remainder(topi.reshape(-1)[src[:n].long()], n_local).to(torch.int32))
    recv = torch.empty_like(send)
    recv_e = torch.empty_like(e_loc)
    dist.all_to_all_single(recv, send, group=ep.handle)
    dist.all_to_all_single(recv_e, e_loc, group=ep.handle)
    ones = torch.ones(P * C, 1, dtype=torch.float32, device=dev)
    y = local_experts(recv, ones, recv_e.view(-1, 1), w13, w2, 0, n_local)  # padding rows -> 0
    back = torch.empty_like(y)
    dist.all_to_all_single(back, y, group=ep.handle)
    y_sorted = back.index_select(0, pos)                                     # dest-sorted order
    return ops.moe_combine(y_sorted, inv, topw)
