"""Device-side expert-parallel dispatch / combine over xGMI peer memory (CL4, config 5).

The DP-attention + EP MoE layer (``parallel/moe.py``) on GPU: every rank exports one
uncached buffer through HIP IPC (handles exchanged once over the process group, as the K15
all-reduce does), and each MoE layer is a handful of kernels (``ops/csrc/ep_exchange.hip``)
that write every routed row straight into its owner's buffer at its final, expert-grouped row,
run the local experts' grouped GEMMs on the received rows, and write the outputs back to the
source slots: exact (no padding rows cross the fabric), no host synchronisation, hipGraph
capturable (epochs live on the device).  The old padded RCCL ``all_to_all_single`` pair stays
the CPU (gloo) reference path.

Parity with the reference: the reference has no expert parallelism; this is
the north-star row CL4 / K12-K14, replacing the stock Seldon runtime selected
at /root/reference/mlflow_operator.py:198,213.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class EPExchange:
    def __init__(self, rank: int, world: int, num_experts: int, top_k: int, hidden: int, max_tokens: int,
                 device, group=None):
        from .. import ops

        ops.load()
        self.rank, self.world, self.group = rank, world, group
        self.E, self.k, self.H, self.tcap = num_experts, top_k, hidden, int(max_tokens)
        self.n_local = num_experts // world
        self.device = torch.device(device)
        self.h = torch.ops.mlop.ep_create(rank, world, num_experts, top_k, hidden, self.tcap,
                                          self.device.index or 0)
        mine = bytes(torch.ops.mlop.ep_ipc_handle(self.h).numpy().tobytes())
        allh = [None] * world
        if world > 1:
            dist.all_gather_object(allh, mine, group=group)
        else:
            allh = [mine]
        table = torch.frombuffer(bytearray(b"".join(allh)), dtype=torch.uint8).view(world, 64).clone()
        torch.ops.mlop.ep_open(self.h, table)
        if world > 1:
            dist.barrier(group=group)

    def dispatch(self, x: torch.Tensor, topi: torch.Tensor, cap_tokens: int):
        """This rank's routed rows to their experts' owners; returns (xp, offsets): the rows this
        rank received, grouped by its local experts ([world * cap * k, H], only the first
        offsets[-1] valid), and the int32 group offsets for the grouped GEMM.  ``cap_tokens``:
        the largest T of any rank in this step (the group agrees on it)."""
        cap = max(int(cap_tokens), x.shape[0])
        xp = torch.empty(self.world * cap * self.k, self.H, dtype=x.dtype, device=x.device)
        offsets = torch.empty(self.n_local + 1, dtype=torch.int32, device=x.device)
        torch.ops.mlop.ep_dispatch(self.h, xp, offsets, x.contiguous(), topi.to(torch.int32).contiguous())
        return xp, offsets

    def combine(self, y: torch.Tensor, topw: torch.Tensor, topi: torch.Tensor, T: int) -> torch.Tensor:
        """Expert outputs back to their sources; out[t] = sum_j topw[t, j] * y_j(t)."""
        out = torch.empty(T, self.H, dtype=y.dtype, device=y.device)
        torch.ops.mlop.ep_combine(self.h, out, y, topw.float().contiguous(), topi.to(torch.int32).contiguous())
        return out

    @property
    def uncached(self) -> bool:
        return bool(torch.ops.mlop.ep_mem_mode(self.h))

    def error(self) -> int:
        """Non-zero: a flag wait timed out (1) or a peer overflowed the agreed capacity (2)."""
        return int(torch.ops.mlop.ep_error(self.h))

    def close(self):
        if self.h:
            torch.ops.mlop.ep_destroy(self.h)
            self.h = 0
