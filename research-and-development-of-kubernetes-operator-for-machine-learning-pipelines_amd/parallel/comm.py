"""Process-group plumbing: one process per GPU, ``torch.distributed`` over RCCL.

On ROCm the ``"nccl"`` backend IS RCCL (xGMI peer links inside a node); CPU
tests use ``"gloo"`` with the same code.  A ``ParallelState`` carries the
tensor-parallel (TP) and expert-parallel (EP) groups of one serving replica;
data-parallel replicas (DP, the reference's per-predictor ``replicas`` /
traffic split) are independent engines and share nothing.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


def env_rank_info():
    """(rank, local_rank, world_size) from torchrun-style env vars (defaults: single process)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def init_distributed(backend: str | None = None, timeout_s: int = 600) -> bool:
    """Initialise the default process group from env (MASTER_ADDR defaults to 127.0.0.1)."""
    rank, local_rank, world = env_rank_info()
    if world <= 1 or dist.is_initialized():
        return dist.is_initialized()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    kw = {}
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
        kw["device_id"] = torch.device("cuda", local_rank)
    dist.init_process_group(backend=backend, rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return True


@dataclass
class Group:
    """A communicator: rank/size within it plus the torch group handle (None = world)."""

    rank: int = 0
    size: int = 1
    handle: object = None
    car: object = None  # CustomAllReduce (K15) for small bf16 messages on GPU
    ex: object = None   # EPExchange (ep_ipc.py): the DP-attention + EP MoE exchange on GPU
    car_status: str = "off"  # K15: "ok" (self-check passed), "fallback" (failed: RCCL / gloo), "off"
    car_check: dict = None   # this rank's K15 start-up self-check verdict (custom_ar.self_check)

    def all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        if self.size > 1:
            if self.car is not None and self.car.eligible(x):
                return self.car.all_reduce(x)
            dist.all_reduce(x, group=self.handle)
        return x

    def all_reduce_add(self, x: torch.Tensor, residual: torch.Tensor) -> torch.Tensor:
        """residual = bf16(residual + bf16(all_reduce(x))) in place (x may be overwritten): one
        K15 launch when eligible, else the all-reduce and the add with the same rounding."""
        if self.size > 1 and self.car is not None and self.car.can_all_reduce_add(x, residual):
            return self.car.all_reduce_add(x, residual)
        self.all_reduce(x)
        residual.copy_((residual.float() + x.float()).to(residual.dtype))
        return residual

    def all_gather(self, x: torch.Tensor, dim: int = -1) -> torch.Tensor:
        if self.size == 1:
            return x
        if self.car is not None and self.car.can_all_gather(x):
            parts = self.car.all_gather(x.contiguous())
            return torch.cat(list(parts.unbind(0)), dim=dim)
        parts = [torch.empty_like(x) for _ in range(self.size)]
        dist.all_gather(parts, x.contiguous(), group=self.handle)
        return torch.cat(parts, dim=dim)

    def all_to_all_single(self, out: torch.Tensor, inp: torch.Tensor, out_splits=None, in_splits=None):
        if self.size == 1:
            out.copy_(inp)
            return out
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.handle)
        return out

    def broadcast(self, x: torch.Tensor, src_rank_in_group: int = 0) -> torch.Tensor:
        if self.size > 1:
            if self.car is not None and self.car.can_broadcast(x):
                return self.car.broadcast(x, src_rank_in_group)
            src = dist.get_global_rank(self.handle, src_rank_in_group) if self.handle is not None else src_rank_in_group
            dist.broadcast(x, src=src, group=self.handle)
        return x

    def barrier(self):
        if self.size > 1:
            dist.barrier(group=self.handle)


@dataclass
class ParallelState:
    tp: Group
    ep: Group
    ep_cpu: object = None  # gloo group over the EP ranks: per-step control (engine.EPSync)
    tp_cpu: object = None  # gloo group over the TP ranks: the step header (engine.StepSync)

    @property
    def tp_size(self) -> int:
        return self.tp.size

    @property
    def tp_rank(self) -> int:
        return self.tp.rank


def single() -> ParallelState:
    return ParallelState(tp=Group(), ep=Group())


def make_parallel_state(tp_size: int = 1, ep_size: int = 1, custom_ar: bool = True) -> ParallelState:
    """Split the world into consecutive TP groups (TP inside a node: xGMI is point-to-point,
    keep TP degree <= 8).  EP reuses the TP ranks (experts sharded over the same GPUs).
    On GPU the TP group gets the K15 one-shot all-reduce for decode-size messages
    (``MLOP_CUSTOM_AR=0`` keeps everything on RCCL)."""
    if not dist.is_initialized():
        assert tp_size == 1 and ep_size == 1, "TP/EP > 1 needs torch.distributed"
        return single()
    world, rank = dist.get_world_size(), dist.get_rank()
    assert world % tp_size == 0, f"world {world} not divisible by tp {tp_size}"
    assert world % ep_size == 0, f"world {world} not divisible by ep {ep_size}"

    def groups(size):  # consecutive blocks of `size` ranks; every rank creates every group
        mine = None
        for start in range(0, world, size):
            ranks = list(range(start, start + size))
            h = dist.new_group(ranks) if size < world else None
            if rank in ranks:
                mine = h
        return mine

    tp_handle = groups(tp_size)
    tp = Group(rank=rank % tp_size, size=tp_size, handle=tp_handle)
    # EP over the TP ranks (tokens replicated by TP attention, partial MoE outputs summed by
    # the TP all-reduce) or over its own block of ranks (all-to-all dispatch / combine)
    ep = tp if ep_size == tp_size else Group(rank=rank % ep_size, size=ep_size, handle=groups(ep_size))
    ep_cpu = None
    if ep_size > 1 and tp_size == 1:  # DP attention + EP: a CPU group for the per-step agreement
        for start in range(0, world, ep_size):
            ranks = list(range(start, start + ep_size))
            h = dist.new_group(ranks, backend="gloo")
            if rank in ranks:
                ep_cpu = h
    tp_cpu = None
    if tp_size > 1:  # the per-step header travels host to host, ahead of the device work
        for start in range(0, world, tp_size):
            ranks = list(range(start, start + tp_size))
            h = dist.new_group(ranks, backend="gloo")
            if rank in ranks:
                tp_cpu = h
    car_env = os.environ.get("MLOP_CUSTOM_AR", "1")
    backend_ok = dist.get_backend(tp_handle) == "nccl" or car_env == "force"  # force: gloo + GPU tests
    if custom_ar and tp_size in (2, 4, 8) and torch.cuda.is_available() and backend_ok and car_env != "0":
        from .custom_ar import CustomAllReduce

        car = CustomAllReduce(tp.rank, tp_size, torch.device("cuda", torch.cuda.current_device()),
                              group=tp_handle)
        # first contact: K15 must reproduce the exact rank-order sum of seeded inputs on EVERY
        # rank before it carries a single real message; otherwise the whole group stays on the
        # process-group collectives (custom_ar.py self_check / agree)
        inj = os.environ.get("MLOP_INJECT_CAR_CORRUPT", "")
        # every rank mapped every peer (else nobody launches a kernel a peer cannot answer)
        if car.agree({"ok": car.init_error is None}):
            verdict = car.self_check(inject_rank=int(inj) if inj.strip() else None)
        else:
            verdict = {"ok": False, "checks": {}, "error_word": -1,
                       "exception": car.init_error or "a peer could not map the IPC buffers"}
        tp.car_check = verdict
        if car.agree(verdict):  # collective: every rank calls it exactly once
            tp.car, tp.car_status = car, "ok"
        else:
            import sys

            print(f"[comm] K15 self-check failed on the TP group (rank {tp.rank}: {verdict}): "
                  "falling back to the process-group collectives", file=sys.stderr, flush=True)
            car.close()
            tp.car_status = "fallback"
    return ParallelState(tp=tp, ep=ep, ep_cpu=ep_cpu, tp_cpu=tp_cpu)


class HostChannel:
    """One-producer / N-consumer broadcast of small int64 messages between the processes of a
    group on ONE node, over POSIX shared memory (``ops/csrc/shm_channel.cc``): the TP leader's
    step header reaches the workers in about a microsecond instead of a gloo TCP broadcast.
    Collective construction over ``cpu_group`` (the segment's name travels once); the name is
    unlinked as soon as every rank mapped it, so a crash leaves nothing in /dev/shm."""

    SLOTS = 64

    class Unavailable(RuntimeError):
        """Raised on EVERY rank of the group when any rank could not create or map the channel
        (callers fall back to gloo together)."""

    def __init__(self, cpu_group, words: int = 16):
        import uuid

        self.words = words
        self.h = 0
        self.rank = dist.get_rank(cpu_group)
        self.size = dist.get_world_size(cpu_group)
        name, err = None, ""
        if self.rank == 0:
            name = f"/mlop-chan-{uuid.uuid4().hex[:16]}"
            try:
                self.h = self._create(name)
            except Exception as e:  # noqa: BLE001 - agreed on below, every rank falls back
                err, name = f"{type(e).__name__}: {e}", None
        box = [name]
        dist.broadcast_object_list(box, src=dist.get_global_rank(cpu_group, 0), group=cpu_group)
        if self.rank != 0:
            if box[0] is None:
                err = "the leader could not create the channel"
            else:
                try:
                    self.h = self._open(box[0])
                except Exception as e:  # noqa: BLE001
                    err = f"{type(e).__name__}: {e}"
        # every rank's verdict (and a barrier: nobody unlinks before all have mapped)
        ok = torch.tensor([0 if err else 1], dtype=torch.int64)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=cpu_group)
        if self.rank == 0 and name is not None:
            torch.ops.mlop.chan_unlink(name)
        if not int(ok.item()):
            self.close()
            raise HostChannel.Unavailable(err or "another rank could not map the channel")
        self._buf = torch.zeros(words, dtype=torch.int64)

    def _create(self, name: str) -> int:
        from .. import ops

        ops.load()
        return torch.ops.mlop.chan_create(name, self.SLOTS, self.size - 1)

    def _open(self, name: str) -> int:
        from .. import ops

        ops.load()
        return torch.ops.mlop.chan_open(name)

    def send(self, vals: torch.Tensor, timeout_s: float = 600.0) -> None:
        import time

        t0 = time.monotonic()
        while not torch.ops.mlop.chan_send(self.h, vals, 20000):
            if time.monotonic() - t0 > timeout_s:
                raise TimeoutError("host channel: consumers stopped reading")

    def recv(self, out: torch.Tensor, timeout_s: float = 3600.0) -> torch.Tensor:
        """Blocks (250 ms slices; the op runs without the GIL) until the next message arrives.
        Inside a slice the native wait spins, yields, then sleeps (shm_channel.cc wait_until),
        so a parked worker of an idle predictor costs ~1 % of a core, not a whole one."""
        import time

        t0 = time.monotonic()
        while not torch.ops.mlop.chan_recv(self.h, self.rank - 1, out, 250000):
            if time.monotonic() - t0 > timeout_s:
                raise TimeoutError("host channel: no message from the producer")
        return out

    def close(self):
        if getattr(self, "h", 0):
            torch.ops.mlop.chan_close(self.h, False)
            self.h = 0


class HostAllGather:
    """Lock-step all-gather of small int64 messages between the processes of a group on ONE node,
    over POSIX shared memory (``ops/csrc/shm_allgather.cc``): the expert-parallel serving loop's
    per-iteration control (request broadcast, output gather, the step agreement) in one
    shared-memory hop each instead of gloo TCP round trips.  Every rank calls ``exchange`` the
    same number of times in the same order; each contributes up to ``max_words`` words and gets
    every rank's words back.  Collective construction over ``cpu_group`` with the same agreement
    as ``HostChannel``: every rank gets the segment, or every rank raises ``Unavailable``
    (``make_host_allgather`` then falls back to gloo on all of them)."""

    SLOTS = 2
    Unavailable = HostChannel.Unavailable

    def __init__(self, cpu_group, max_words: int):
        import uuid

        self.max_words = int(max_words)
        self.h = 0
        self.rank = dist.get_rank(cpu_group)
        self.size = dist.get_world_size(cpu_group)
        name, err = None, ""
        if self.rank == 0:
            name = f"/mlop-xg-{uuid.uuid4().hex[:16]}"
            try:
                self.h = self._create(name)
            except Exception as e:  # noqa: BLE001 - agreed on below
                err, name = f"{type(e).__name__}: {e}", None
        box = [name]
        dist.broadcast_object_list(box, src=dist.get_global_rank(cpu_group, 0), group=cpu_group)
        if self.rank != 0:
            if box[0] is None:
                err = "the leader could not create the segment"
            else:
                try:
                    self.h = self._open(box[0])
                except Exception as e:  # noqa: BLE001
                    err = f"{type(e).__name__}: {e}"
        ok = torch.tensor([0 if err else 1], dtype=torch.int64)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=cpu_group)
        if self.rank == 0 and name is not None:
            torch.ops.mlop.chan_unlink(name)
        if not int(ok.item()):
            self.close()
            raise HostAllGather.Unavailable(err or "another rank could not map the segment")
        self._out = torch.zeros(self.size, self.max_words, dtype=torch.int64)
        self._counts = torch.zeros(self.size, dtype=torch.int64)

    def _create(self, name: str) -> int:
        from .. import ops

        ops.load()
        return torch.ops.mlop.xg_create(name, self.size, self.SLOTS, self.max_words)

    def _open(self, name: str) -> int:
        from .. import ops

        ops.load()
        return torch.ops.mlop.xg_open(name, self.rank)

    def exchange(self, vals: torch.Tensor, timeout_s: float = 600.0) -> list:
        """Every rank's int64 words, in rank order (views into a reused buffer: copy what must
        outlive the next exchange).  Waits in 250 ms slices (the op runs without the GIL and
        resumes where it stopped); a peer silent for ``timeout_s`` raises TimeoutError."""
        import time

        vals = vals.contiguous()
        t0 = time.monotonic()
        while not torch.ops.mlop.xg_exchange(self.h, vals, self._out, self._counts, 250000):
            if time.monotonic() - t0 > timeout_s:
                raise TimeoutError("host all-gather: a peer stopped exchanging (dead rank?)")
        return [self._out[q, :int(self._counts[q])] for q in range(self.size)]

    def close(self):
        if getattr(self, "h", 0):
            torch.ops.mlop.xg_close(self.h)
            self.h = 0


class GlooAllGather:
    """``HostAllGather``'s API over the gloo group (two collectives: the counts, then the words
    padded to the longest): the fallback when shared memory is unavailable (ranks on different
    hosts, no /dev/shm)."""

    def __init__(self, cpu_group, max_words: int):
        self.group, self.max_words = cpu_group, int(max_words)
        self.size = dist.get_world_size(cpu_group)

    def exchange(self, vals: torch.Tensor, timeout_s: float = 600.0) -> list:
        n = torch.tensor([vals.numel()], dtype=torch.int64)
        ns = [torch.zeros(1, dtype=torch.int64) for _ in range(self.size)]
        dist.all_gather(ns, n, group=self.group)
        m = max(int(x) for x in ns)
        if m == 0:
            return [torch.zeros(0, dtype=torch.int64) for _ in range(self.size)]
        buf = torch.zeros(m, dtype=torch.int64)
        buf[:vals.numel()] = vals
        parts = [torch.zeros(m, dtype=torch.int64) for _ in range(self.size)]
        dist.all_gather(parts, buf, group=self.group)
        return [p[:int(c)] for p, c in zip(parts, ns)]

    def close(self):
        pass


def make_host_allgather(cpu_group, max_words: int):
    """The shared-memory all-gather when every rank can map it, else ``GlooAllGather``; decided
    collectively.  (The gloo form measured the same EP = 2 serving rate on one GPU:
    profiles/r05_ep_control.md.)"""
    import sys

    try:
        return HostAllGather(cpu_group, max_words)
    except HostAllGather.Unavailable as e:
        print(f"[comm] shared-memory all-gather unavailable ({e}): gloo", file=sys.stderr)
    return GlooAllGather(cpu_group, max_words)
