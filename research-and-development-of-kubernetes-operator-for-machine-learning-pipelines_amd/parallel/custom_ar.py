"""K15 custom one-shot all-reduce over xGMI peer memory (``ops/csrc/allreduce.hip``).

Tensor-parallel decode all-reduces small [B, hidden] bf16 tensors twice per
layer; RCCL's ring pays 2(N-1) latency-bound hops for them.  Here every rank
exports one device buffer through HIP IPC, the ranks exchange the 64-byte
handles once over the (RCCL or gloo) process group, and each call is ONE
kernel in which every rank reads all peers' inputs in a single hop across the
point-to-point xGMI links, with an epoch-flag handshake (system-scope
release / acquire) instead of a collective library call.  The kernel keeps its
epochs on the device, so it is captured into the decode hipGraphs like any
other op.  Messages above ``max_bytes`` (prefill) stay on RCCL.

Parity with the reference: the reference has no collective at all (SURVEY.md
§2.2-2.3); this implements the north-star row K15 / CL1.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

# registered buffer per parity: one-shot messages up to this size, two-shot ones up to half of it
# (tensor-parallel prefill chunks: 8192 x 4096 bf16 = 64 MiB at Llama-3-70B TP 8, chunked below)
DEFAULT_MAX_BYTES = 64 << 20
# above this message size the two-shot kernel (reduce-scatter + all-gather, each one hop over the
# full mesh: 2 (N-1)/N x the message per rank instead of the one-shot's N-1 x)
TWO_SHOT_MIN_BYTES = 512 << 10


# data parities in their own cached buffer, flags alone uncached (allreduce.hip "Memory").  Off
# by default: one uncached buffer measured the same at the two-shot sizes (1-64 MiB, -5..+9 %)
# and 11-23 % faster at 256 KiB-4 MiB one-shot messages (scripts/bench_car.py,
# profiles/r05_car_memory.md)
SPLIT_DATA = False


class CustomAllReduce:
    def __init__(self, rank: int, world: int, device, group=None, max_bytes: int = DEFAULT_MAX_BYTES,
                 split_data: bool | None = None):
        from .. import ops

        ops.load()
        self.rank, self.world, self.group = rank, world, group
        self.device = torch.device(device)
        self.max_bytes = int(max_bytes)
        self.split_data = SPLIT_DATA if split_data is None else bool(split_data)
        self.h = torch.ops.mlop.car_create(rank, world, self.max_bytes, self.device.index or 0, self.split_data)
        mine = torch.ops.mlop.car_ipc_handle(self.h)
        if world > 1:
            allh = [None] * world
            dist.all_gather_object(allh, bytes(mine.numpy().tobytes()), group=group)
        else:
            allh = [bytes(mine.numpy().tobytes())]
        table = torch.frombuffer(bytearray(b"".join(allh)), dtype=torch.uint8).view(world, 128).clone()
        torch.ops.mlop.car_open(self.h, table)
        if world > 1:
            dist.barrier(group=group)

    def eligible(self, x: torch.Tensor) -> bool:
        if not (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and x.numel() % 8 == 0):
            return False
        n = 2 * x.numel()
        return n <= self.max_bytes if n < TWO_SHOT_MIN_BYTES else 2 * n <= self.max_bytes

    def all_reduce(self, x: torch.Tensor, out: torch.Tensor | None = None, two_shot: bool | None = None) -> torch.Tensor:
        """Sum over ranks (rank order, fp32 accumulation: identical on every rank).  One-shot
        below TWO_SHOT_MIN_BYTES, two-shot above (``two_shot`` forces either); in place when
        ``out`` is None."""
        out = x if out is None else out
        if two_shot is None:
            two_shot = 2 * x.numel() >= TWO_SHOT_MIN_BYTES
        torch.ops.mlop.car_all_reduce(self.h, out, x, bool(two_shot))
        return out

    def can_all_reduce_add(self, x: torch.Tensor, residual: torch.Tensor) -> bool:
        return (self.eligible(x) and 2 * x.numel() < TWO_SHOT_MIN_BYTES and residual.is_contiguous()
                and residual.dtype == x.dtype and residual.numel() == x.numel()
                and residual.data_ptr() != x.data_ptr())

    def all_reduce_add(self, x: torch.Tensor, residual: torch.Tensor) -> torch.Tensor:
        """residual = bf16(residual + bf16(sum over ranks of x)) in ONE one-shot launch (the
        tensor-parallel decode norm chain: the residual add rides in the all-reduce)."""
        torch.ops.mlop.car_all_reduce_add(self.h, residual, x)
        return residual

    def can_broadcast(self, x: torch.Tensor) -> bool:
        n = x.numel() * x.element_size()
        return x.is_cuda and x.is_contiguous() and n % 16 == 0 and n <= self.max_bytes

    def broadcast(self, x: torch.Tensor, root: int = 0) -> torch.Tensor:
        """In-place broadcast from group rank ``root``: ONE kernel; every other rank copies the
        root's bytes straight out of its IPC buffer (one xGMI hop, no host round trip, no RCCL
        launch).  Shares the per-block epochs with the all-reduce kernels."""
        torch.ops.mlop.car_broadcast(self.h, x, int(root))
        return x

    def can_all_gather(self, x: torch.Tensor) -> bool:
        n = x.numel() * x.element_size()
        return x.is_cuda and x.is_contiguous() and n % 4 == 0 and 0 < n <= self.max_bytes

    def all_gather(self, x: torch.Tensor) -> torch.Tensor:
        """[world, *x.shape] of every rank's ``x`` in rank order: ONE kernel, each peer's piece
        read straight from its IPC buffer (the TP vocab-parallel logits / greedy pairs)."""
        out = torch.empty((self.world,) + tuple(x.shape), dtype=x.dtype, device=x.device)
        torch.ops.mlop.car_all_gather(self.h, out, x)
        return out

    @property
    def uncached(self) -> bool:
        """True when the flag buffer is uncached device memory (allreduce.hip)."""
        return bool(torch.ops.mlop.car_mem_mode(self.h) & 1)

    @property
    def data_cached(self) -> bool:
        """True when the data parities live in their own ordinary (cached) buffer."""
        return bool(torch.ops.mlop.car_mem_mode(self.h) & 2)

    def error(self) -> int:
        """Non-zero if any call timed out waiting for a peer (the result is then invalid)."""
        return int(torch.ops.mlop.car_error(self.h))

    def close(self):
        if self.h:
            torch.ops.mlop.car_destroy(self.h)
            self.h = 0
