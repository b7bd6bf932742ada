"""Tensor-parallel row-parallel projections with the all-reduce overlapped (config 4, large M).

A Megatron row-parallel projection (O, down) leaves a partial [M, H] sum on every rank; the
layer then all-reduces it and runs residual add + RMSNorm before the next column-parallel GEMM.
Issued as one GEMM -> one all-reduce -> one norm, the device sits idle on the fabric for the
whole all-reduce (Llama-3-70B TP=8 at M = 4096: 64 MiB per all-reduce, 160 per forward).  Here
M is cut into row chunks: chunk i's GEMM runs on the compute stream while chunk i-1's all-reduce
(K15 two-shot kernel over xGMI peer memory, or RCCL) and its add + RMSNorm run on a
communication stream, so only the last chunk's all-reduce + norm is exposed.  Same result bit
for bit as the unchunked order (rows are independent in all three ops).

Decode sizes (M below ``MIN_ROWS``, inside the captured graphs) keep the single-chunk order.
"""
from __future__ import annotations

import contextlib
import os

import torch

from .. import ops

MIN_ROWS = 1024
CHUNK_ROWS = 1024  # a multiple of the GEMM's 256-row tile
_COMM: dict = {}


def comm_stream(device) -> torch.cuda.Stream:
    d = torch.device(device)
    i = d.index if d.index is not None else torch.cuda.current_device()
    s = _COMM.get(i)
    if s is None:
        s = _COMM[i] = torch.cuda.Stream(device=torch.device("cuda", i))
    return s


def chunks_of(M: int, chunk: int = CHUNK_ROWS, align: int = 256):
    """Row ranges of about ``chunk`` rows (at least 2), each a multiple of ``align`` rows but the last."""
    if chunk <= 0:
        return [(0, M)]
    n = max(2, (M + chunk - 1) // chunk)
    per = max(align, ((M + n - 1) // n + align - 1) // align * align)
    return [(lo, min(M, lo + per)) for lo in range(0, M, per)]


def row_parallel_add_norm(a: torch.Tensor, w: torch.Tensor, tp, residual: torch.Tensor, norm_w: torch.Tensor,
                          eps: float, chunk: int | None = None, min_rows: int | None = None) -> torch.Tensor:
    """x = rmsnorm(residual += all_reduce(a @ w^T)) * norm_w, residual updated in place.  On CPU
    (gloo tests) the chunks run in order on the one stream: same arithmetic, no overlap."""
    M, N = a.shape[0], w.shape[0]
    cuda = a.is_cuda
    chunk = CHUNK_ROWS if chunk is None else chunk
    min_rows = MIN_ROWS if min_rows is None else min_rows
    parts = [(0, M)]
    if cuda:
        # a chunk must still fill the chip: >= one 256 x 256 tile per CU (256 tiles), else its
        # GEMM runs on part of the GPU and the overlap costs more than it hides (measured on one
        # GPU, scripts/tp_overlap_trace.py: 1024-row chunks of a N = 8192 projection, 128 tiles
        # each, 311 vs 196 us per call)
        fill = (256 * 256 * 256 + N - 1) // N
        chunk = max(chunk, (fill + 255) // 256 * 256)
        min_rows = max(min_rows, 2 * chunk)
    if tp.size > 1 and M >= min_rows and not (cuda and torch.cuda.is_current_stream_capturing()):
        parts = chunks_of(M, chunk)
    if len(parts) == 1:
        o = ops.gemm(a, w)
        tp.all_reduce(o)
        return ops.add_rmsnorm(o, residual, norm_w, eps)
    o = torch.empty(M, N, dtype=a.dtype, device=a.device)
    x = torch.empty_like(o)
    if cuda:
        cur = torch.cuda.current_stream(a.device)
        comm = comm_stream(a.device)
        comm.wait_stream(cur)  # residual / norm weights and earlier work are ready
    for lo, hi in parts:
        ops.gemm(a[lo:hi], w, out=o[lo:hi])
        if cuda:
            ev = torch.cuda.Event()
            ev.record(cur)
            ctx = torch.cuda.stream(comm)
            comm.wait_event(ev)
        else:
            ctx = contextlib.nullcontext()
        with ctx:
            tp.all_reduce(o[lo:hi])
            ops.add_rmsnorm(o[lo:hi], residual[lo:hi], norm_w, eps, out=x[lo:hi])
    if cuda:
        cur.wait_stream(comm)
    return x
