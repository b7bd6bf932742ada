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
        # First contact never raises half-way: a rank whose buffer or peer mapping fails records
        # it (init_error) and still takes part in every collective below, so the group reaches
        # the self-check agreement together (a raise here would leave the peers blocked in the
        # handle exchange or the barrier)
        self.h, self.init_error = 0, None
        mine = None
        try:
            self.h = torch.ops.mlop.car_create(rank, world, self.max_bytes, self.device.index or 0, self.split_data)
            mine = bytes(torch.ops.mlop.car_ipc_handle(self.h).numpy().tobytes())
        except Exception as e:  # noqa: BLE001 - agreed on in make_parallel_state
            self.init_error = f"create: {type(e).__name__}: {e}"
        if world > 1:
            allh = [None] * world
            dist.all_gather_object(allh, mine, group=group)
        else:
            allh = [mine]
        if self.init_error is None and any(h is None for h in allh):
            self.init_error = "a peer could not create its buffer"
        if self.init_error is None:
            try:
                table = torch.frombuffer(bytearray(b"".join(allh)), dtype=torch.uint8).view(world, 128).clone()
                torch.ops.mlop.car_open(self.h, table)
            except Exception as e:  # noqa: BLE001
                self.init_error = f"open: {type(e).__name__}: {e}"
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
            try:
                torch.ops.mlop.car_destroy(self.h)
            finally:
                self.h = 0

    # ------------------------------------------------------------ first contact --
    def self_check(self, hidden: int = 4096, inject_rank: int | None = None) -> dict:
        """Start-up agreement test of the IPC peers, run by EVERY rank of the group before the
        first real call: a peer mapping that reads stale / wrong memory (a cross-device
        coherence or dmabuf bug) would otherwise serve garbage at full speed, since the only
        runtime guard (``error``) catches a dead peer, not a wrong sum.

        Every rank generates every rank's input from a seed (rank r: seed 0x5EED + r), so the
        exact expected result is known locally without trusting any collective: the fp32 sum
        in rank order rounded to bf16 -- what the kernels compute, bit for bit.  Checked: the
        process-group all-reduce of the one-shot inputs (fp32, within its own rounding; a
        cross-check of the fallback path itself, run first), then one-shot (16 rows), two-shot
        (256 rows, above TWO_SHOT_MIN_BYTES), the one-shot all-reduce + residual add, the
        broadcast and the all-gather.  ``inject_rank``: that rank perturbs its one-shot output (the
        forced-corruption test, env ``MLOP_INJECT_CAR_CORRUPT``).  Returns this rank's
        verdict; ``agree`` makes it the group's."""
        dev, W = self.device, self.world
        rows = {"one_shot": 16, "two_shot": max(16, (TWO_SHOT_MIN_BYTES // (2 * hidden)) * 2)}

        def inputs(n, salt):
            xs = []
            for p in range(W):
                g = torch.Generator(device=dev).manual_seed(0x5EED + 7919 * salt + p)
                xs.append(torch.randn(n, hidden, device=dev, generator=g).to(torch.bfloat16))
            return xs

        def oracle(xs):
            acc = torch.zeros(xs[0].shape, dtype=torch.float32, device=dev)
            for x in xs:  # rank order, fp32: the kernels' accumulation
                acc += x.float()
            return acc

        res = {"ok": True, "checks": {}}
        if self.init_error is not None:  # nothing to test: this rank never mapped its peers
            return {"ok": False, "checks": {}, "exception": self.init_error, "error_word": -1}
        try:
            # the process-group path the fallback would use, FIRST: it is the only blocking
            # collective here, so every rank reaches it even if a K15 call below raises on one
            # rank (the K15 kernels' spins are bounded: the peers then see the error word and
            # everyone meets again in ``agree``)
            xs = inputs(rows["one_shot"], 0)
            exp = oracle(xs)
            pg = xs[self.rank].float()
            if dist.is_initialized() and W > 1:
                on_cpu = dist.get_backend(self.group) == "gloo"
                t = pg.cpu() if on_cpu else pg
                dist.all_reduce(t, group=self.group)
                pg = t.to(dev)
            res["checks"]["process_group"] = bool(torch.allclose(pg, exp, rtol=1e-5, atol=1e-5 * W))
            for salt, (name, n) in enumerate(rows.items()):
                xs = inputs(n, salt)
                out = torch.empty_like(xs[self.rank])
                self.all_reduce(xs[self.rank].clone(), out, two_shot=(name == "two_shot"))
                if inject_rank == self.rank and name == "one_shot":
                    out.view(-1)[0] += 1.0
                exp = oracle(xs)
                res["checks"][name] = bool(torch.equal(out, exp.to(torch.bfloat16)))
                if name == "one_shot":
                    resid = xs[(self.rank + 1) % W].clone()  # any residual both sides know
                    want = (resid.float() + exp.to(torch.bfloat16).float()).to(torch.bfloat16)
                    self.all_reduce_add(xs[self.rank].clone(), resid)
                    res["checks"]["all_reduce_add"] = bool(torch.equal(resid, want))
                    b = xs[self.rank].clone()
                    self.broadcast(b, 0)
                    res["checks"]["broadcast"] = bool(torch.equal(b, xs[0]))
                    ga = self.all_gather(xs[self.rank])
                    res["checks"]["all_gather"] = bool(torch.equal(ga, torch.stack(xs)))
            torch.cuda.synchronize(dev)
            res["error_word"] = self.error()
        except Exception as e:  # noqa: BLE001 - reported, the group falls back together
            res["exception"] = f"{type(e).__name__}: {e}"
            res["error_word"] = -1
        res["ok"] = (res["error_word"] == 0 and bool(res["checks"])
                     and all(v for k, v in res["checks"].items() if k != "process_group"))
        return res

    def agree(self, verdict: dict) -> bool:
        """Every rank's self-check verdict -> the group's (MIN over ranks, on the host group when
        the process group is gloo, else a device tensor over RCCL): the whole group keeps K15 or
        the whole group falls back, never a mix (a rank on K15 would wait forever for a peer
        that posts nothing)."""
        if self.world == 1 or not dist.is_initialized():
            return bool(verdict["ok"])
        on_cpu = dist.get_backend(self.group) == "gloo"
        t = torch.tensor([1 if verdict["ok"] else 0], dtype=torch.int64,
                         device="cpu" if on_cpu else self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return bool(int(t.item()))
