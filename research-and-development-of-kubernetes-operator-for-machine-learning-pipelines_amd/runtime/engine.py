"""Continuous-batching inference engine (G5) with hipGraph-captured decode (G1).

One engine per model replica (DP replica = one engine; a TP replica runs one
engine per rank in lock-step, rank 0 owning the scheduler and broadcasting
step metadata).

Step policy:
  * prefill steps pack up to ``max_num_batched_tokens`` prompt tokens of
    admitted requests (chunked: a long prompt spans several steps);
  * decode steps run every running sequence, one token each, replaying the
    hipGraph captured for the smallest batch bucket >= B (padded rows attend to
    nothing), so a decode step costs one graph launch + one metadata H2D + one
    token D2H;
  * prompt work is scheduled when requests wait and either nothing is decoding,
    enough requests are queued (``prefill_min_batch``) or the oldest has waited
    ``max_decode_gap`` decode steps (bounded TTFT without fragmenting decode);
    while sequences decode it runs as a MIXED step (``mixed_prefill``): every
    running row's decode token plus prompt chunks up to the token budget in one
    eager ragged forward, so decode rides in the prefill's larger-M GEMMs
    instead of stalling behind a separate prefill pass;
  * KV pages come from a free-list; on exhaustion the newest running sequence
    is preempted (pages freed, recomputed later).
"""
from __future__ import annotations

import collections
import itertools
import operator
import os
import sys
import time
from dataclasses import dataclass, field
from enum import Enum

import numpy as np
import torch

from .. import ops
from .attn_meta import MetaBuffers, plan_partitions
from .kv_cache import BLOCK_SIZE, BlockAllocator, KVCache, blocks_for_budget, blocks_needed, prefix_hashes
from .sampler import Sampler, SamplingParams
from .tracing import StepTracer, TorchProfileWindow


KIND_STOP, KIND_EAGER, KIND_GRAPH, KIND_BARRIER = 0, 1, 2, 3


class StepSync:
    """Lock-step execution across a tensor-parallel group.  Rank 0 alone
    schedules.  Per step it sends two things:

      * the step header [kind, T, num_tiles, n_logits, part_tokens, nparts, bucket,
        num_flash_tiles, greedy] HOST to host, over the TP group's gloo (CPU) group: a worker
        learns what step t+1 is while the device still runs step t, so it enqueues step t+1's
        forward (and its graph replay) ahead, exactly as the leader does under one-step-ahead
        scheduling, and no worker ever reads a device tensor back to decide what to run;
      * the step's packed metadata buffer (attn_meta.MetaBuffers: int32 metadata, ids and
        logits index in ONE device buffer, already uploaded by one H2D, decode ids gathered on
        the device from the previous step's tokens) as ONE in-stream device broadcast of its
        used prefix (header word 9: up to the highest block-table row in use): the K15 IPC
        broadcast kernel on GPU (parallel/custom_ar.py: each worker copies the leader's bytes in
        one hop, no host round trip), RCCL / gloo otherwise, ordered after the previous forward
        on every rank's stream.
    STOP / BARRIER steps carry the header only."""

    NHDR = 10

    def __init__(self, group, cpu_group=None):
        import os

        self.g = group
        self.cpu = cpu_group
        self.is_leader = group.rank == 0
        self.hdr = torch.zeros(self.NHDR, dtype=torch.int64)
        # the header's host path: the native shared-memory channel (TP groups live on one node),
        # gloo's broadcast as the fallback (the channel cannot be built on every rank)
        self.chan = None
        if cpu_group is not None:
            from ..parallel.comm import HostChannel

            try:  # collective: every rank gets a channel, or every rank raises and uses gloo
                self.chan = HostChannel(cpu_group, words=self.NHDR)
            except HostChannel.Unavailable as e:
                print(f"[engine] TP step-header channel unavailable ({e}): gloo broadcast", file=sys.stderr)
                self.chan = None

    def _bcast_header(self):
        import torch.distributed as dist

        if self.cpu is None:  # no host group (single process): nothing to agree on
            return
        if self.chan is not None:
            if self.is_leader:
                self.chan.send(self.hdr)
            else:
                self.chan.recv(self.hdr)
            return
        dist.broadcast(self.hdr, src=dist.get_global_rank(self.cpu, 0), group=self.cpu)

    def send(self, eng, kind, T, nt, nl, part, nparts, bucket, npt=0, greedy=0):
        n = eng.meta.extent(eng.rows_hi)
        self.hdr[:] = torch.tensor([kind, T, nt, nl, part, nparts, bucket, npt, greedy, n], dtype=torch.int64)
        self._bcast_header()
        if kind not in (KIND_STOP, KIND_BARRIER):
            self.g.broadcast(eng.meta.dbuf[:n], 0)

    def recv(self, eng):
        self._bcast_header()
        hdr = tuple(self.hdr.tolist())
        if hdr[0] not in (KIND_STOP, KIND_BARRIER):
            self.g.broadcast(eng.meta.dbuf[:hdr[9]], 0)
        return hdr[:9]


class _Tokens:
    """Token ids chosen inside ``_execute`` (TP greedy: no logits were gathered)."""

    __slots__ = ("ids",)

    def __init__(self, ids):
        self.ids = ids

    def __getitem__(self, k):
        return _Tokens(self.ids[k])


class EPSync:
    """Lock-step agreement of a data-parallel-attention / expert-parallel group (config 5, CL4).

    Every rank schedules its OWN requests, but each MoE layer is an all-to-all over the whole
    group, so every rank must run a forward in the same step, with the same MoE capacity, and
    either all replay a decode graph of the same bucket or all run eager.  Once per step every
    rank calls ``agree``: [has_work, wants_eager, tokens, bucket, busy] from every rank over the
    group's shared-memory all-gather (parallel/comm.py ``HostAllGather``: one host hop, no GPU
    sync; gloo when shared memory is unavailable), reduced by MAX on each rank -> what the whole
    group does this step.  A rank with nothing to do joins with a padding-only forward."""

    def __init__(self, group, cpu_group):
        from ..parallel.comm import make_host_allgather

        self.g, self.cpu = group, cpu_group
        self.last_any = 1
        self.last_busy = 1
        self.xg = make_host_allgather(cpu_group, 8)
        self._v = torch.zeros(5, dtype=torch.int64)

    def agree(self, has_work: int, eager: int, tokens: int, bucket: int, busy: int = 1):
        """``busy``: this rank still holds requests (queued, running or in flight) even if it
        launches nothing this step; the group is done only when no rank is busy."""
        v = self._v
        v[0], v[1], v[2], v[3], v[4] = has_work, eager, tokens, bucket, busy
        rows = self.xg.exchange(v)
        any_work, any_eager, t_max, b_max, any_busy = torch.stack(rows).max(dim=0).values.tolist()
        self.last_any, self.last_busy = any_work, any_busy
        return any_work, any_eager, t_max, b_max


class Status(Enum):
    WAITING = 0
    PREFILL = 1
    RUNNING = 2
    FINISHED = 3


@dataclass
class Sequence:
    seq_id: int
    prompt: list
    params: SamplingParams
    output: list = field(default_factory=list)
    blocks: list = field(default_factory=list)
    row: int = -1
    num_cached: int = 0
    status: Status = Status.WAITING
    arrival: float = field(default_factory=time.perf_counter)
    first_token_time: float | None = None
    finish_time: float | None = None
    finish_reason: str | None = None
    hashes: list = field(default_factory=list)  # prefix hashes of this sequence's full pages
    n_reg: int = 0                              # leading pages matched in / registered to the prefix cache

    @property
    def length(self) -> int:
        return len(self.prompt) + len(self.output)

    def token_at(self, i: int) -> int:
        n = len(self.prompt)
        return self.prompt[i] if i < n else self.output[i - n]

    def tokens(self, a: int, b: int):
        n = len(self.prompt)
        if b <= n:
            return self.prompt[a:b]
        if a >= n:
            return self.output[a - n:b - n]
        return list(self.prompt[a:]) + self.output[:b - n]


@dataclass
class EngineConfig:
    max_num_seqs: int = 256
    max_num_batched_tokens: int = 8192
    max_model_len: int = 4096
    num_kv_blocks: int | None = None       # None: size from kv_cache_bytes / free HBM
    kv_cache_bytes: int | None = None
    gpu_memory_utilization: float = 0.90
    kv_fraction: float = 0.5  # pages for this share of max_num_seqs x max_model_len (mean context;
                              # preemption covers the tail) - same policy as controller/placement.py
    use_graphs: bool = True
    graph_buckets: tuple = (1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024)
    prefill_min_batch: int = 1
    max_decode_gap: int = 0
    mixed_prefill: bool = True    # prefill chunks ride in the decode step (one forward)
    mixed_min_chunk: int = 64     # below this many free token slots, decode alone
    seed: int = 0
    enable_prefix_caching: bool = True  # share computed prompt pages between requests (same prefix)
    # one-step-ahead scheduling (TP = EP = 1, mixed prefill): step t+1 is built and launched
    # while step t still runs on the device; step t's tokens are read back afterwards
    async_scheduling: bool = True


@dataclass
class StepOutput:
    seq_id: int
    token: int
    finished: bool
    finish_reason: str | None = None


class _ParamsList(list):
    pass


class _AllGreedy:
    """Stands in for a list of greedy SamplingParams of any length."""

    all_greedy = True

    def __getitem__(self, k):
        return self


_ALL_GREEDY = _AllGreedy()


class StepBatch:
    """One step's outputs as arrays (no per-token Python objects on the hot path);
    iterating yields ``StepOutput`` lazily."""

    __slots__ = ("seq_ids", "tokens", "fin", "reasons")

    def __init__(self, seq_ids, tokens, fin, reasons: dict):
        self.seq_ids, self.tokens, self.fin, self.reasons = seq_ids, tokens, fin, reasons

    @classmethod
    def from_list(cls, outs: list):
        return cls(np.array([o.seq_id for o in outs], dtype=np.int64),
                   np.array([o.token for o in outs], dtype=np.int64),
                   np.array([o.finished for o in outs], dtype=bool),
                   {o.seq_id: o.finish_reason for o in outs if o.finished})

    def __len__(self):
        return len(self.seq_ids)

    def __iter__(self):
        for sid, tok, f in zip(self.seq_ids.tolist(), self.tokens.tolist(), self.fin.tolist()):
            yield StepOutput(sid, tok, f, self.reasons.get(sid) if f else None)

    @property
    def finished(self) -> list:
        return [StepOutput(int(self.seq_ids[i]), int(self.tokens[i]), True, self.reasons.get(int(self.seq_ids[i])))
                for i in np.nonzero(self.fin)[0]]


class Engine:
    def __init__(self, model, cfg: EngineConfig | None = None):
        self.model = model
        self.checkpoint_dir = None  # set by deploy.build_engine when the weights came from a checkpoint
        self.cfg = cfg = cfg or EngineConfig()
        self.device = model.device
        mc = model.cfg
        self.max_model_len = min(cfg.max_model_len, mc.max_position)
        nb = cfg.num_kv_blocks or self._auto_blocks()
        tp = model.ps.tp
        self.step_sync = StepSync(tp, model.ps.tp_cpu) if tp.size > 1 else None
        ep = model.ps.ep
        self.ep_sync = EPSync(ep, model.ps.ep_cpu) if (tp.size == 1 and ep.size > 1) else None
        if tp.size > 1:  # every rank must address the same page ids: agree on the minimum
            t = torch.tensor([nb], dtype=torch.int64, device=self.device)
            import torch.distributed as dist

            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=tp.handle)
            nb = int(t.item())
        t_kv = time.perf_counter()
        # TP ranks must all hold every page id the leader hands out: eager backing there
        self.kv = KVCache(mc.num_layers, nb, model.n_kv, mc.head_dim, self.device, model.dtype,
                          lazy=False if tp.size > 1 else None)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        kv_alloc_ms = int(1e3 * (time.perf_counter() - t_kv))
        self.alloc = BlockAllocator(nb, available=self.kv.ready_blocks())
        self.max_blocks_per_seq = blocks_needed(self.max_model_len)
        self.buckets = sorted(b for b in cfg.graph_buckets if b <= cfg.max_num_seqs) or [cfg.max_num_seqs]
        if self.buckets[-1] < cfg.max_num_seqs:
            self.buckets.append(cfg.max_num_seqs)
        self.G = model.n_q // model.n_kv
        self.meta = MetaBuffers(max(cfg.max_num_batched_tokens, cfg.max_num_seqs),
                                cfg.max_num_seqs + self.buckets[-1], self.max_blocks_per_seq,
                                self.G, model.n_kv, self.max_model_len, self.device)
        self.free_rows = list(range(cfg.max_num_seqs - 1, -1, -1))
        self.rows_hi = 0  # high-water row + 1: the block-table rows a step's upload / broadcast moves
        # struct-of-arrays state of running rows: the decode hot path is vectorised
        R = cfg.max_num_seqs
        self.r_len = np.zeros(R, np.int64)      # tokens in the sequence (prompt + output)
        self.r_gen = np.zeros(R, np.int64)      # generated tokens
        self.r_maxgen = np.zeros(R, np.int64)
        self.r_last = np.zeros(R, np.int64)     # last token (next decode input)
        self.r_ignore = np.zeros(R, bool)       # ignore_eos
        self.r_hasstop = np.zeros(R, bool)      # has stop_token_ids (checked in Python)
        self.r_nblk = np.zeros(R, np.int64)     # KV pages held
        self.r_sid = np.zeros(R, np.int64)
        self.r_random = np.zeros(R, bool)       # non-greedy sampling
        self.r_epoch = np.zeros(R, np.int64)    # bumped when a row is released (async: stale results)
        self.r_tokidx = np.zeros(R, np.int64)   # async: the row's pending token in the in-flight step
        # rows of ``self.running`` in order, and their output lists (kept in step with the
        # list: appended rows go to ``_rows_add``, finished rows are masked out in
        # ``_decode_finish``, a preempted one popped off the end; anything else sets dirty)
        self._rows = np.zeros(0, np.int32)
        self._outs: list[list] = []
        self._rows_add: list[int] = []
        self._rows_dirty = True
        self.sampler = Sampler(self.device, cfg.seed)
        self.waiting: collections.deque[Sequence] = collections.deque()
        self.prefilling: list[Sequence] = []
        self.running: list[Sequence] = []
        self.seqs: dict[int, Sequence] = {}
        self._ids = itertools.count()
        self._decode_since_prefill = 0
        self.graphs: dict[int, tuple] = {}
        self.graph_pool = None
        self.stats = collections.Counter()
        # one-step-ahead (async) scheduling state: the in-flight step, its token read-back
        # buffers (two pinned, alternating) and the event after its metadata upload.  Under TP
        # only the leader schedules (workers follow the host-side headers, StepSync); under EP
        # every rank runs it, the per-step agreement happens at launch time (_ep_agree)
        self._async = cfg.async_scheduling and cfg.mixed_prefill
        self._pending = None
        self._ids_gather = None
        self._meta_ev = None
        cuda = self.device.type == "cuda"
        nmax = self.meta.max_tokens
        self._toks_h = [torch.zeros(nmax, dtype=torch.int64, pin_memory=cuda) for _ in range(2)]
        self._toks_flip = 0
        self._src_h = torch.zeros(R, dtype=torch.int64, pin_memory=cuda)
        self._src_d = torch.zeros(R, dtype=torch.int64, device=self.device)
        if self.ep_sync is not None and self.device.type == "cuda":
            self._setup_ep_exchange()
        self.stats["kv_alloc_ms"] = kv_alloc_ms
        self.stats.update(self.kv.timing_ms)
        self.tracer = StepTracer()
        self.profile_window = TorchProfileWindow()
        import os

        # fault injection (canary tests of the GPU-side guards): every forward step also runs a
        # device delay kernel of this many microseconds (ops/csrc/elementwise.hip device_delay)
        self._inject_device_us = int(os.environ.get("MLOP_INJECT_STEP_DEVICE_US", "0") or 0)
        if self._inject_device_us and self.device.type != "cuda":
            self._inject_device_us = 0
        if self._inject_device_us:
            from .. import ops as _ops

            _ops.load()

        # TP decode graphs capture the row-parallel all-reduces (K15 one-shot kernel, or RCCL
        # inside capture); the vocab gather runs after the replay (``_gather``).
        if cfg.use_graphs and self.device.type == "cuda":
            self.capture_graphs()
        self.kv.start_background_fill()  # after capture: the rest of a lazy KV arena
        self.stats["kv_ready_blocks_at_start"] = self.alloc.available

    def _setup_ep_exchange(self):
        """DP-attention + EP on GPU: the device-side MoE exchange over IPC peer memory
        (parallel/ep_ipc.py), sized for the largest forward this engine runs; collective over
        the EP group (every rank builds its engine together).  Without it (CPU): the group's
        all_to_all (parallel/moe.py)."""
        import os

        ep, mc = self.model.ps.ep, self.model.cfg
        if ep.ex is not None or not getattr(mc, "num_experts", 0):
            return
        from ..parallel.ep_ipc import EPExchange

        ep.ex = EPExchange(ep.rank, ep.size, mc.num_experts, mc.top_k, mc.hidden_size, self.meta.max_tokens,
                           self.device, group=ep.handle)

    # ----------------------------------------------------------- sizing --
    def _auto_blocks(self) -> int:
        mc, m = self.model.cfg, self.model
        if self.cfg.kv_cache_bytes:
            budget = self.cfg.kv_cache_bytes
        elif self.device.type == "cuda" and os.environ.get("MLOP_SHARE_GPU", "0") not in ("", "0", "false"):
            # one-GPU rehearsal of a multi-rank pod: the ranks size their pools concurrently, so
            # a "free HBM" reading races the others' allocations; split the card's usable
            # capacity evenly instead (every rank holds a same-size weight shard)
            _, total = torch.cuda.mem_get_info(self.device)
            n = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", 1)))
            usable = total * self.cfg.gpu_memory_utilization - 4 * 2**30 - n * m.weight_bytes()
            budget = int(max(usable / max(1, n), 2**30))
        elif self.device.type == "cuda":
            free, total = torch.cuda.mem_get_info(self.device)
            reserve = total * (1 - self.cfg.gpu_memory_utilization) + 4 * 2**30
            budget = int(max(free - reserve, 2**30))
        else:
            budget = 64 * 2**20
        need = int(self.cfg.kv_fraction * self.cfg.max_num_seqs *
                   blocks_needed(min(self.cfg.max_model_len, mc.max_position))) + 2
        nb = blocks_for_budget(budget, mc.num_layers, m.n_kv, mc.head_dim)
        return int(min(nb, need))

    # -------------------------------------------------------- requests --
    def check_request(self, prompt, params: SamplingParams | None = None) -> None:
        """ValueError when this engine cannot serve the request (empty / too long prompt, token
        ids outside the vocabulary, unusable sampling parameters)."""
        if not prompt:
            raise ValueError("empty prompt")
        if len(prompt) >= self.max_model_len:
            raise ValueError(f"prompt of {len(prompt)} tokens exceeds max_model_len {self.max_model_len}")
        V = self.model.cfg.vocab_size
        if min(prompt) < 0 or max(prompt) >= V:
            raise ValueError(f"prompt token ids must be in [0, {V})")
        (params or SamplingParams()).validate()

    def add_request(self, prompt, params: SamplingParams | None = None, seq_id: int | None = None) -> Sequence:
        params = params or SamplingParams()
        prompt = list(prompt)
        self.check_request(prompt, params)
        sid = next(self._ids) if seq_id is None else seq_id
        seq = Sequence(sid, prompt, params)
        self.seqs[sid] = seq
        self.waiting.append(seq)
        return seq

    def abort(self, seq_id: int) -> None:
        seq = self.seqs.get(seq_id)
        if seq is None or seq.status == Status.FINISHED:
            return
        for lst in (self.prefilling, self.running):
            if seq in lst:
                lst.remove(seq)
        self._rows_dirty = True
        if seq in self.waiting:
            self.waiting.remove(seq)
        self._finish(seq, "abort")

    def has_work(self) -> bool:
        return bool(self.waiting or self.prefilling or self.running or self._pending_alive())

    @property
    def num_running(self) -> int:
        return len(self.running) + len(self.prefilling)

    def kv_usage(self) -> float:
        return self.alloc.usage()

    # ------------------------------------------------------ bookkeeping --
    def _ensure_blocks(self, seq: Sequence, ctx: int) -> bool:
        need = blocks_needed(ctx) - len(seq.blocks)
        if need <= 0:
            return True
        if not self.alloc.can_allocate(need):
            return False
        new = self.alloc.allocate(need)
        start = len(seq.blocks)
        seq.blocks.extend(new)
        self.meta.bt_h[seq.row, start:start + need] = new
        self.r_nblk[seq.row] = len(seq.blocks)
        return True

    def _release(self, seq: Sequence):
        if seq.blocks:
            self.alloc.free(seq.blocks)
            seq.blocks = []
        seq.n_reg = 0
        if seq.row >= 0:
            self.r_nblk[seq.row] = 0
            self.r_epoch[seq.row] += 1  # an in-flight step's result for this row is stale
            self.free_rows.append(seq.row)
            seq.row = -1
        seq.num_cached = 0

    def _params_of_running(self):
        """Sampling params of the decode batch; a falsy ``any_random`` lets the sampler
        take the all-greedy fast path without a per-sequence Python scan."""
        lst = _ParamsList(s.params for s in self.running) if self.r_random[self._sync_rows()].any() else _ALL_GREEDY
        return lst

    def _register_running(self, s: Sequence):
        r, p = s.row, s.params
        self.r_random[r] = not p.greedy
        self.r_len[r], self.r_gen[r], self.r_maxgen[r] = s.length, len(s.output), p.max_tokens
        self.r_last[r] = s.output[-1] if s.output else s.prompt[-1]
        self.r_ignore[r], self.r_hasstop[r], self.r_sid[r] = p.ignore_eos, bool(p.stop_token_ids), s.seq_id
        self._rows_add.append(r)  # s was just appended to self.running

    def _finish(self, seq: Sequence, reason: str):
        seq.status = Status.FINISHED
        seq.finish_reason = reason
        seq.finish_time = time.perf_counter()
        self._release(seq)

    def _preempt(self, seq: Sequence):
        self.stats["preemptions"] += 1
        self._release(seq)
        seq.status = Status.WAITING
        self.waiting.appendleft(seq)

    # ------------------------------------------------------- scheduling --
    def _want_prefill(self) -> bool:
        if self.prefilling:
            return True
        if not self.waiting or not self.free_rows:
            return False
        if not self.running:
            return True
        c = self.cfg
        return (len(self.waiting) >= c.prefill_min_batch
                or (c.max_decode_gap and self._decode_since_prefill >= c.max_decode_gap))

    def step(self) -> list[StepOutput]:
        """One scheduler step (traced: ``self.tracer`` spans, optional torch.profiler window)."""
        self.profile_window.before_step()
        t0 = time.perf_counter()
        n0d, n0p = self.stats["decode_tokens"], self.stats["prefill_tokens"]
        kind, out = self._step()
        self._check_peers()
        self.tracer.record(kind, t0, time.perf_counter(), decode_tokens=self.stats["decode_tokens"] - n0d,
                           prefill_tokens=self.stats["prefill_tokens"] - n0p, running=len(self.running),
                           waiting=len(self.waiting))
        self.profile_window.after_step()
        return out

    def _check_peers(self):
        """Error words of the device-side collectives (K15 all-reduce / broadcast / all-gather, the
        EP exchange; host-mapped, so this is a plain load, no sync): a flag wait that timed out
        means a peer rank died or wedged and its results are garbage.  Fail loudly -- the launcher
        restarts the predictor -- instead of serving them."""
        ps = getattr(self.model, "ps", None)
        if ps is None:
            return
        for name, obj in (("tensor-parallel custom collectives", getattr(ps.tp, "car", None)),
                          ("expert-parallel exchange", getattr(getattr(ps, "ep", None), "ex", None))):
            code = obj.error() if obj is not None else 0
            if code:
                raise RuntimeError(f"{name}: a peer flag wait timed out (error word {code}): a rank died "
                                   f"or wedged, results since then are invalid")

    def _step(self):
        self._launched = False
        kind, out = self._step_local()
        if self.ep_sync is not None and not self._launched:
            self._ep_idle()  # nothing launched here (idle, or nothing schedulable): still join
        return kind, out

    def _ep_idle(self):
        """EP rank with nothing scheduled: agree, then run a padding-only forward (one row
        that attends nothing) eagerly, or replay the agreed decode graph on padding rows."""
        any_work, eager, t_max, bucket = self.ep_sync.agree(0, 0, 0, 0, int(self.has_work()))
        if not any_work:
            return
        self._wait_meta()  # async: the previous step's metadata H2D must have read the host buffer
        empty = np.zeros(0, dtype=np.int32)
        if eager or bucket not in self.graphs:
            self.meta.fill_decode(empty, empty, np.zeros(0, dtype=np.int64), pad_to=1)
            self.meta.upload(1, 1, self.rows_hi)
            self.model.moe_capacity_tokens = t_max
            self.model.forward(self.meta.ids_d[:1], self.meta.meta(1, 1, 1, 32, 1), self.kv)
        else:
            self.meta.fill_decode(empty, empty, np.zeros(0, dtype=np.int64), pad_to=bucket)
            self.meta.upload(bucket, bucket, self.rows_hi)
            self.graphs[bucket][0].replay()
        if self._async and self.device.type == "cuda":
            self._meta_ev = torch.cuda.Event()
            self._meta_ev.record()
        self.stats["ep_idle_steps"] += 1

    def _step_local(self):
        if self.alloc.available < self.alloc.num_blocks and not self.kv.fill_failed:
            self.alloc.grow(self.kv.ready_blocks())  # lazily backed KV chunks became ready
            if self.kv.fill_failed:
                self.stats["kv_fill_failed"] = 1
                self.stats["kv_blocks_backed"] = self.alloc.available
        if self._async and (self._pending is not None or self.running):
            return self._async_step()
        if self._want_prefill():
            if self.running and self.cfg.mixed_prefill:
                kind, out = "mixed", self._mixed_step()
            else:
                kind, out = "prefill", self._prefill_step()
            if out is not None:
                self._decode_since_prefill = 0
                return kind, out
        if self.running:
            self._decode_since_prefill += 1
            return "decode", self._decode_step()
        return "idle", []

    # ---------------------------------------------------------- prefill --
    def _collect_prefill(self, budget: int):
        """Admit prompt chunks up to ``budget`` tokens: continuing chunked
        prefills first, then waiting requests (each needs a free row + pages)."""
        batch, chunks = [], []
        for seq in list(self.prefilling):
            if budget <= 0:
                break
            n = min(seq.length - seq.num_cached, budget)
            if not self._ensure_blocks(seq, seq.num_cached + n):
                break
            batch.append(seq)
            chunks.append(n)
            budget -= n
        while budget > 0 and self.waiting and self.free_rows:
            seq = self.waiting[0]
            seq.row = self.free_rows.pop()
            self.rows_hi = max(self.rows_hi, seq.row + 1)
            if self.cfg.enable_prefix_caching:
                self._match_prefix(seq)
            n = min(seq.length - seq.num_cached, budget)
            if not self._ensure_blocks(seq, seq.num_cached + n):
                self._release(seq)  # matched prefix pages back to the cache, row freed
                break
            self.waiting.popleft()
            # prefix-cache stats once per admission (a head request that waits for pages
            # re-matches every step and must not inflate the hit rate)
            self.stats["prefix_query_tokens"] += seq.length
            self.stats["prefix_hit_tokens"] += seq.num_cached
            seq.status = Status.PREFILL
            self.prefilling.append(seq)
            batch.append(seq)
            chunks.append(n)
            budget -= n
        return batch, chunks

    def _match_prefix(self, seq: Sequence) -> None:
        """Reuse cached pages of this sequence's longest cached prefix (never the page
        holding its last token: that one is computed to get the next-token logits)."""
        nfull = (seq.length - 1) // BLOCK_SIZE
        if nfull <= 0:
            return
        if len(seq.hashes) < nfull:
            prev = seq.hashes[-1] if seq.hashes else b""
            seq.hashes += prefix_hashes(seq.tokens(0, nfull * BLOCK_SIZE), nfull, len(seq.hashes), prev)
        m = 0
        for h in seq.hashes[:nfull]:
            b = self.alloc.lookup(h)
            if b is None:
                break
            self.alloc.take(b)
            seq.blocks.append(b)
            m += 1
        if m:
            self.meta.bt_h[seq.row, :m] = seq.blocks
            self.r_nblk[seq.row] = m
            seq.num_cached = m * BLOCK_SIZE
            seq.n_reg = m

    def _register_prefix(self, seq: Sequence, ctx: int) -> None:
        """Publish the pages this prefill filled (full pages of computed tokens)."""
        full = ctx // BLOCK_SIZE
        if full <= seq.n_reg:
            return
        if len(seq.hashes) < full:
            prev = seq.hashes[-1] if seq.hashes else b""
            seq.hashes += prefix_hashes(seq.tokens(0, full * BLOCK_SIZE), full, len(seq.hashes), prev)
        for i in range(seq.n_reg, full):
            self.alloc.register(seq.blocks[i], seq.hashes[i])
        seq.n_reg = full

    def _prefill_finish(self, batch, ctx, done, tokens) -> list:
        outs = []
        ti = 0
        for s, c, d in zip(batch, ctx, done):
            s.num_cached = c
            if self.cfg.enable_prefix_caching:
                self._register_prefix(s, c)
            if d:
                self.prefilling.remove(s)
                s.status = Status.RUNNING
                self.running.append(s)
                o = self._append(s, tokens[ti])
                if not o.finished:
                    self._register_running(s)
                outs.append(o)
                ti += 1
        return outs

    def _prefill_step(self):
        batch, chunks = self._collect_prefill(self.cfg.max_num_batched_tokens)
        if not batch:
            return None
        rows = [s.row for s in batch]
        ctx = [s.num_cached + n for s, n in zip(batch, chunks)]
        toks = [s.tokens(s.num_cached, c) for s, c in zip(batch, ctx)]
        done = [c == s.length for s, c in zip(batch, ctx)]
        T, nt, nl = self.meta.fill(rows, chunks, ctx, toks, want_logits=done)
        part, nparts = plan_partitions(nt, self.model.n_kv, max(ctx))
        done_params = [s.params for s, d in zip(batch, done) if d]
        logits = self._launch(KIND_EAGER, T, nt, nl, part, nparts, 0,
                              greedy=all(p.greedy for p in done_params))
        tokens = None
        if nl:
            tokens = self._sample(logits, done_params,
                                  lambda: [len(s.output) for s, d in zip(batch, done) if d]).tolist()
        else:
            torch.cuda.synchronize() if self.device.type == "cuda" else None
        self.stats["prefill_steps"] += 1
        self.stats["prefill_tokens"] += T
        return StepBatch.from_list(self._prefill_finish(batch, ctx, done, tokens))

    # ------------------------------------------------------------ mixed --
    def _mixed_step(self):
        """Decode every running sequence AND prefill prompt chunks in ONE eager
        forward (chunked-prefill piggybacking): the decode rows share the
        prefill's weight reads and its larger-M GEMMs instead of paying a
        separate M=B pass; the ragged paged-attention kernel takes both kinds
        of tile.  Returns None (caller decodes alone) when nothing fits."""
        t0 = time.perf_counter()
        rows, ctx_d = self._decode_rows()
        B = len(rows)
        budget = self.cfg.max_num_batched_tokens - B
        if B == 0 or budget < self.cfg.mixed_min_chunk:
            return None
        batch, chunks = self._collect_prefill(budget)
        if not batch:
            return None
        p_rows = [s.row for s in batch]
        p_ctx = [s.num_cached + n for s, n in zip(batch, chunks)]
        p_toks = [s.tokens(s.num_cached, c) for s, c in zip(batch, p_ctx)]
        done = [c == s.length for s, c in zip(batch, p_ctx)]
        T, nt, nl = self.meta.fill_mixed(rows, ctx_d.astype(np.int32), self.r_last[rows],
                                         p_rows, chunks, p_ctx, p_toks, want_logits=done)
        part, nparts = plan_partitions(nt, self.model.n_kv, max(int(ctx_d.max()), max(p_ctx)))
        t1 = time.perf_counter()
        done_seqs = [s for s, d in zip(batch, done) if d]
        dparams = self._params_of_running()
        if getattr(dparams, "all_greedy", False) and all(s.params.greedy for s in done_seqs):
            params = _ALL_GREEDY
        else:
            params = _ParamsList([s.params for s in self.running] + [s.params for s in done_seqs])
        logits = self._launch(KIND_EAGER, T, nt, nl, part, nparts, 0,
                              greedy=getattr(params, "all_greedy", False))
        toks = self._sample(logits, params, lambda: self._gen_index(rows, done_seqs)).cpu().numpy().astype(np.int64)
        t2 = time.perf_counter()
        self.stats["mixed_steps"] += 1
        self.stats["decode_tokens"] += B
        self.stats["prefill_tokens"] += T - B
        d_out = self._decode_finish(rows, toks[:B])
        p_out = self._prefill_finish(batch, p_ctx, done, toks[B:].tolist())
        self.stats["mixed_host_us"] += int(1e6 * (t1 - t0 + time.perf_counter() - t2))
        self.stats["mixed_device_us"] += int(1e6 * (t2 - t1))
        if not p_out:
            return d_out
        p = StepBatch.from_list(p_out)
        reasons = dict(d_out.reasons)
        reasons.update(p.reasons)
        return StepBatch(np.concatenate([d_out.seq_ids, p.seq_ids]), np.concatenate([d_out.tokens, p.tokens]),
                         np.concatenate([d_out.fin, p.fin]), reasons)

    # ------------------------------------------------- async scheduling --
    # Step t+1 is built from the scheduler state as it stands after step t's LAUNCH: every
    # running row decodes again (a row whose step-t token turns out to be EOS / a stop token
    # is computed once more and its result dropped), its input id is gathered on the device
    # from step t's sampled tokens, and lengths / page needs are advanced at launch time (they
    # do not depend on token values).  Step t's tokens are read back (pinned copy + event,
    # so the read waits for step t only, never for the step queued behind it) and applied
    # after step t+1 is queued: the host's bookkeeping and the next step's preparation run
    # while the device computes, and the device never waits for the host between steps.
    # A row's results are stale once it was released (finish, abort, preemption): r_epoch.

    def _pending_alive(self) -> bool:
        p = self._pending
        if p is None:
            return False
        rows, ep = p["rows"], p["epochs"]
        return bool(len(rows)) and bool((self.r_epoch[rows] == ep).any())

    def _wait_meta(self):
        """The previous step's metadata H2D has executed: the host buffers may be rewritten."""
        ev, self._meta_ev = self._meta_ev, None
        if ev is not None:
            ev.synchronize()

    def _async_step(self):
        prev, self._pending = self._pending, None
        if not self.running:
            # nothing decodes: finish the in-flight step (its finished rows free their slots),
            # then this step's prompt work runs as a synchronous prefill step
            out = self._async_post(prev) if prev is not None else StepBatch.from_list([])
            if self._want_prefill():
                p = self._prefill_step()
                if p is not None and len(p):
                    self._decode_since_prefill = 0
                    reasons = dict(out.reasons)
                    reasons.update(p.reasons)
                    out = StepBatch(np.concatenate([out.seq_ids, p.seq_ids]), np.concatenate([out.tokens, p.tokens]),
                                    np.concatenate([out.fin, p.fin]), reasons)
                    return "prefill", out
                if p is not None:
                    return "prefill", out
            return "idle", out
        kind, pend = "idle", None
        if self.running:
            self._wait_meta()
            if self._want_prefill():
                pend = self._async_launch(prev, mixed=True)
                if pend is not None:
                    kind = "mixed"
                    self._decode_since_prefill = 0
            if pend is None:
                self._decode_since_prefill += 1
                pend = self._async_launch(prev, mixed=False)
                kind = "decode" if pend is not None else kind
        self._pending = pend
        out = self._async_post(prev) if prev is not None else StepBatch.from_list([])
        return kind, out

    def _async_launch(self, prev, mixed: bool):
        """Build, launch and advance one step; returns its pending record (None: nothing to run)."""
        t0 = time.perf_counter()
        rows, ctx_d = self._decode_rows()
        B = len(rows)
        if B == 0:
            return None
        ctx_d = ctx_d.astype(np.int32)
        batch, chunks = [], []
        if mixed:
            budget = self.cfg.max_num_batched_tokens - B
            if budget < self.cfg.mixed_min_chunk:
                return None
            batch, chunks = self._collect_prefill(budget)
            if not batch:
                return None
        # decode input ids: on the device from the in-flight step, else the host's last token
        gather = prev is not None and prev.get("toks_d") is not None
        last = np.zeros(B, np.int64) if gather else self.r_last[rows]
        dparams = self._params_of_running()
        greedy = getattr(dparams, "all_greedy", False)
        if mixed:
            p_rows = [s.row for s in batch]
            p_ctx = [s.num_cached + n for s, n in zip(batch, chunks)]
            p_toks = [s.tokens(s.num_cached, c) for s, c in zip(batch, p_ctx)]
            done = [c == s.length for s, c in zip(batch, p_ctx)]
            T, nt, nl = self.meta.fill_mixed(rows, ctx_d, last, p_rows, chunks, p_ctx, p_toks, want_logits=done)
            part, nparts = plan_partitions(nt, self.model.n_kv, max(int(ctx_d.max()), max(p_ctx)))
            done_seqs = [s for s, d in zip(batch, done) if d]
            if greedy and all(s.params.greedy for s in done_seqs):
                params = _ALL_GREEDY
            else:
                params = _ParamsList([s.params for s in self.running] + [s.params for s in done_seqs])
            launch = (KIND_EAGER, T, nt, nl, part, nparts, 0)
            greedy = getattr(params, "all_greedy", False)
        else:
            done_seqs = []
            params = dparams
            bucket = next((b for b in self.buckets if b >= B), None)
            if bucket is not None and self.graphs.get(bucket) is not None:
                self.meta.fill_decode(rows, ctx_d, last, pad_to=bucket)
                self._repad = (rows, ctx_d, last, int(ctx_d.max()))  # EP: the group may re-pad it
                launch = (KIND_GRAPH, bucket, bucket, bucket, 0, 0, bucket)
            else:
                self.meta.fill_decode(rows, ctx_d, last, pad_to=B)
                part, nparts = plan_partitions(B, self.model.n_kv, int(ctx_d.max()))
                launch = (KIND_EAGER, B, B, B, part, nparts, 0)
        if gather:
            self._src_h[:B].copy_(torch.from_numpy(self.r_tokidx[rows]))
            self._ids_gather = (B, prev["toks_d"])
        t1 = time.perf_counter()
        logits = self._launch(*launch, greedy=greedy)
        if launch[0] == KIND_GRAPH:
            logits = logits[:B]
        toks_d = self._sample(logits, params, lambda: self._gen_index(rows, done_seqs))
        n = int(toks_d.shape[0])
        toks_h = self._toks_h[self._toks_flip][:n]
        self._toks_flip ^= 1
        ev = None
        if self.device.type == "cuda":
            toks_h.copy_(toks_d, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:
            toks_h.copy_(toks_d)
        # advance what does not depend on token values: decode rows gained a token (pending)
        seqs_d = list(self.running)  # aligned with rows (_decode_rows synced them)
        self.r_len[rows] += 1
        self.r_gen[rows] += 1
        self.r_tokidx[rows] = np.arange(B)
        self.stats["decode_tokens"] += B
        if mixed:
            self.stats["mixed_steps"] += 1
            self.stats["prefill_tokens"] += T - B
            self._prefill_advance(batch, p_ctx, done, B)
        elif launch[0] == KIND_GRAPH:
            self.stats["graph_steps"] += 1
            self.stats["decode_steps"] += 1
        else:
            self.stats["eager_decode_steps"] += 1
            self.stats["decode_steps"] += 1
        snap_rows = np.concatenate([rows, np.asarray([s.row for s in done_seqs], dtype=rows.dtype)])
        pend = {"rows": snap_rows, "epochs": self.r_epoch[snap_rows].copy(), "seqs": seqs_d + done_seqs,
                "toks_d": toks_d, "toks_h": toks_h, "ev": ev, "retire": set()}
        self._retire_by_length(pend)
        self.stats["async_host_us"] += int(1e6 * (t1 - t0 + time.perf_counter() - t1))
        return pend

    def _prefill_advance(self, batch, ctx, done, B):
        """Prompt chunks of a launched step: cached lengths, prefix pages, and the sequences
        whose prompt completed join the running rows (their first token is pending)."""
        j = 0
        for s, c, d in zip(batch, ctx, done):
            s.num_cached = c
            if self.cfg.enable_prefix_caching:
                self._register_prefix(s, c)
            if d:
                self.prefilling.remove(s)
                s.status = Status.RUNNING
                self.running.append(s)
                r, p = s.row, s.params
                self.r_random[r] = not p.greedy
                self.r_len[r], self.r_gen[r], self.r_maxgen[r] = s.length + 1, len(s.output) + 1, p.max_tokens
                self.r_ignore[r], self.r_hasstop[r], self.r_sid[r] = p.ignore_eos, bool(p.stop_token_ids), s.seq_id
                self.r_tokidx[r] = B + j
                self._rows_add.append(r)
                j += 1

    def _retire_by_length(self, pend):
        """Rows whose pending token is their last (max_tokens / max_model_len) leave the
        running set now; they finish when that token is applied."""
        rows = self._sync_rows()
        fin = (self.r_gen[rows] >= self.r_maxgen[rows]) | (self.r_len[rows] >= self.max_model_len)
        if not fin.any():
            return
        run = self.running
        fi = np.nonzero(fin)[0]
        pend["retire"] = {run[i].seq_id for i in fi.tolist()}
        keep = np.nonzero(~fin)[0]
        get = operator.itemgetter(*keep.tolist()) if len(keep) > 1 else None
        if len(keep) == 0:
            self.running, self._outs = [], []
        elif len(keep) == 1:
            self.running, self._outs = [run[keep[0]]], [self._outs[keep[0]]]
        else:
            self.running, self._outs = list(get(run)), list(get(self._outs))
        self._rows = rows[keep]

    def _async_post(self, pend) -> StepBatch:
        """Apply an in-flight step's tokens (waits for that step only)."""
        t0 = time.perf_counter()
        if pend["ev"] is not None:
            pend["ev"].synchronize()
        rows = pend["rows"]
        n = len(rows)
        toks = pend["toks_h"][:n].numpy().copy() if n else np.zeros(0, np.int64)
        alive = self.r_epoch[rows] == pend["epochs"]
        if not alive.all():
            ai = np.nonzero(alive)[0]
            rows, toks = rows[ai], toks[ai]
            seqs = [pend["seqs"][i] for i in ai.tolist()]
        else:
            seqs = pend["seqs"]
        if not len(rows):
            return StepBatch.from_list([])
        now = time.perf_counter()
        for s in seqs:
            if s.first_token_time is None:
                s.first_token_time = now
        collections.deque(map(list.append, [s.output for s in seqs], toks.tolist()), maxlen=0)
        self.r_last[rows] = toks
        eos = self.model.cfg.eos_ids
        is_eos = (toks == eos[0]) if len(eos) == 1 else np.isin(toks, eos)
        fin_stop = (~self.r_ignore[rows]) & is_eos
        for i in np.nonzero(self.r_hasstop[rows])[0].tolist():
            if int(toks[i]) in seqs[i].params.stop_token_ids:
                fin_stop[i] = True
        retire = pend["retire"]
        fin_len = np.zeros(len(rows), bool)
        if retire:
            fin_len = np.fromiter((s.seq_id in retire for s in seqs), dtype=bool, count=len(seqs))
        fin = fin_stop | fin_len
        sids = self.r_sid[rows].copy()
        reasons = {}
        fi = np.nonzero(fin)[0]
        if len(fi):
            done = [seqs[i] for i in fi.tolist()]
            stopped = set()
            for i, s in zip(fi.tolist(), done):
                reasons[s.seq_id] = "stop" if fin_stop[i] else "length"
                if s.seq_id not in retire:
                    stopped.add(s.seq_id)
            if stopped:  # still in the running set (speculatively decoding again)
                self.running = [s for s in self.running if s.seq_id not in stopped]
                self._rows_dirty = True
            for s in done:
                self._finish(s, reasons[s.seq_id])
        self.stats["async_host_us"] += int(1e6 * (time.perf_counter() - t0))
        return StepBatch(sids, toks, fin, reasons)

    # ----------------------------------------------------------- decode --
    def _decode_rows(self):
        """Rows of the running batch with a KV slot for their next token: only rows
        crossing a page boundary allocate (vectorised test, Python only for those
        few); on exhaustion the newest sequence is preempted."""
        while True:
            rows = self._sync_rows()
            ctx = self.r_len[rows]
            nblk = self.r_nblk[rows]
            want = (ctx + BLOCK_SIZE - 1) // BLOCK_SIZE
            need = np.nonzero(want > nblk)[0]
            if len(need) and self.alloc.can_allocate(len(need)) and (want[need] - nblk[need] == 1).all():
                # the steady-state case, vectorised: each crossing row takes exactly one page
                new = self.alloc.allocate(len(need))
                r = rows[need]
                self.meta.bt_h[r, nblk[need]] = new
                self.r_nblk[r] += 1
                run = self.running
                collections.deque(map(list.append, [run[i].blocks for i in need.tolist()], new), maxlen=0)
                return rows, ctx
            ok = True
            for i in need.tolist():
                s = self.running[i]
                # the row's length (async: it counts the in-flight step's token, s.length not yet)
                if not self._ensure_blocks(s, int(ctx[i])):
                    self._preempt(self.running.pop())  # newest goes back to the queue
                    self._rows = self._rows[:-1]
                    self._outs.pop()
                    ok = False
                    break
            if ok:
                return rows, ctx

    def _sync_rows(self) -> np.ndarray:
        """``self._rows`` brought in step with ``self.running`` (O(appended) per step; a
        full rebuild only after an out-of-band change such as an abort)."""
        if self._rows_dirty:
            run = self.running
            self._rows = np.fromiter((s.row for s in run), dtype=np.int32, count=len(run))
            self._outs = [s.output for s in run]
            self._rows_add.clear()
            self._rows_dirty = False
        elif self._rows_add:
            n = len(self._rows_add)
            self._rows = np.concatenate([self._rows, np.asarray(self._rows_add, dtype=np.int32)])
            self._outs.extend(s.output for s in self.running[-n:])
            self._rows_add.clear()
        return self._rows

    def _decode_step(self):
        t0 = time.perf_counter()
        rows, ctx = self._decode_rows()
        B = len(rows)
        if B == 0:
            return StepBatch.from_list([])
        ctx = ctx.astype(np.int32)
        last = self.r_last[rows]
        bucket = next((b for b in self.buckets if b >= B), None)
        g = self.graphs.get(bucket) if bucket is not None else None
        params = self._params_of_running()
        greedy = getattr(params, "all_greedy", False)
        if g is not None:
            self.meta.fill_decode(rows, ctx, last, pad_to=bucket)
            self._repad = (rows, ctx, last, int(ctx.max()))
            t1 = time.perf_counter()
            logits = self._launch(KIND_GRAPH, bucket, bucket, bucket, 0, 0, bucket, greedy=greedy)[:B]
            self.stats["graph_steps"] += 1
        else:
            self.meta.fill_decode(rows, ctx, last, pad_to=B)
            part, nparts = plan_partitions(B, self.model.n_kv, int(ctx.max()))
            t1 = time.perf_counter()
            logits = self._launch(KIND_EAGER, B, B, B, part, nparts, 0, greedy=greedy)
            self.stats["eager_decode_steps"] += 1
        toks = self._sample(logits, params, lambda: self._gen_index(rows, ())).cpu().numpy().astype(np.int64)
        t2 = time.perf_counter()
        self.stats["decode_steps"] += 1
        self.stats["decode_tokens"] += B
        outs = self._decode_finish(rows, toks)
        t3 = time.perf_counter()
        # host-side cost accounting (us): prep before launch, device (launch..tokens), bookkeeping
        self.stats["decode_host_prep_us"] += int(1e6 * (t1 - t0))
        self.stats["decode_device_us"] += int(1e6 * (t2 - t1))
        self.stats["decode_host_post_us"] += int(1e6 * (t3 - t2))
        return outs

    def _decode_finish(self, rows, toks) -> StepBatch:
        """Vectorised bookkeeping of one decode token per running row."""
        self.r_len[rows] += 1
        self.r_gen[rows] += 1
        self.r_last[rows] = toks
        fin_len = (self.r_gen[rows] >= self.r_maxgen[rows]) | (self.r_len[rows] >= self.max_model_len)
        eos = self.model.cfg.eos_ids
        is_eos = (toks == eos[0]) if len(eos) == 1 else np.isin(toks, eos)
        fin_stop = (~self.r_ignore[rows]) & is_eos
        run = self.running
        hs = np.nonzero(self.r_hasstop[rows])[0]
        for i in hs.tolist():
            if int(toks[i]) in run[i].params.stop_token_ids:
                fin_stop[i] = True
        fin = fin_stop | fin_len
        # one token onto every running sequence's output list, at C speed
        collections.deque(map(list.append, self._outs, toks.tolist()), maxlen=0)
        sids = self.r_sid[rows].copy()
        reasons = {}
        fi = np.nonzero(fin)[0]
        if len(fi):
            done = [run[i] for i in fi.tolist()]
            for i, s in zip(fi.tolist(), done):
                reasons[s.seq_id] = "stop" if fin_stop[i] else "length"
            keep = np.nonzero(~fin)[0]
            if len(keep) == 0:
                self.running, self._outs = [], []
            elif len(keep) == 1:
                self.running, self._outs = [run[keep[0]]], [self._outs[keep[0]]]
            else:
                get = operator.itemgetter(*keep.tolist())
                self.running, self._outs = list(get(run)), list(get(self._outs))
            self._rows = rows[keep]
            for s in done:
                self._finish(s, reasons[s.seq_id])
        return StepBatch(sids, toks, fin, reasons)

    def _append(self, s: Sequence, tok: int) -> StepOutput:
        s.output.append(int(tok))
        if s.first_token_time is None:
            s.first_token_time = time.perf_counter()
        p = s.params
        reason = None
        if (not p.ignore_eos and tok in self.model.cfg.eos_ids) or tok in p.stop_token_ids:
            reason = "stop"
        elif len(s.output) >= p.max_tokens:
            reason = "length"
        elif s.length >= self.max_model_len:
            reason = "length"
        if reason:
            if s in self.running:
                self.running.remove(s)
            self._finish(s, reason)
        return StepOutput(s.seq_id, int(tok), reason is not None, reason)

    # --------------------------------------------------------- execution --
    def _launch(self, kind: int, T: int, nt: int, nl: int, part: int, nparts: int, bucket: int,
                greedy: bool = False):
        """Ship this step's metadata to the device and run it.  With tensor
        parallelism, rank 0 (the only rank that schedules) puts the step header in the
        packed metadata buffer and broadcasts it to the TP group in ONE collective
        (SURVEY §2.5 CL5); the other ranks run the same ``_execute`` from ``worker_loop``.
        Returns logits, or (TP, all-greedy rows) the chosen token ids already."""
        self._launched = True
        npt = self.meta.npt  # flash-prefill tiles of the metadata just filled
        if self.ep_sync is not None:
            kind, T, nt, nl, part, nparts, bucket = self._ep_agree(kind, T, nt, nl, part, nparts, bucket)
        self.meta.upload(T, nl, self.rows_hi)
        g = self._ids_gather
        if g is not None:
            # async: decode rows' input ids = the previous (in-flight) step's sampled tokens,
            # gathered on the device after the metadata H2D (which carried placeholders) and
            # before the TP broadcast of the buffer, so the workers receive the real ids
            self._ids_gather = None
            B, toks_d = g
            self._src_d[:B].copy_(self._src_h[:B], non_blocking=True)
            if toks_d.dtype == self.meta.ids_d.dtype and toks_d.dim() == 1:  # one gather kernel, no copy
                torch.index_select(toks_d, 0, self._src_d[:B], out=self.meta.ids_d[:B])
            else:
                self.meta.ids_d[:B].copy_(toks_d.index_select(0, self._src_d[:B]))
        if self.step_sync is not None:
            t0 = time.perf_counter()
            self.step_sync.send(self, kind, T, nt, nl, part, nparts, bucket, npt, int(greedy))
            self.stats["tp_sync_us"] += int(1e6 * (time.perf_counter() - t0))
            self.stats["tp_sync_calls"] += 1
        if self._async and self.device.type == "cuda":
            self._meta_ev = torch.cuda.Event()
            self._meta_ev.record()
        return self._execute(kind, T, nt, nl, part, nparts, bucket, npt, greedy)

    def _ep_agree(self, kind, T, nt, nl, part, nparts, bucket):
        """EP lock-step: the group's common step shape.  Someone eager -> everyone eager, MoE
        capacity = the group's largest token count (a graph-planned decode runs its padded
        rows eagerly); all graph -> everyone replays the largest agreed bucket (re-padded)."""
        any_work, eager, t_max, b_max = self.ep_sync.agree(1, int(kind == KIND_EAGER), T, bucket)
        if eager:
            if kind == KIND_GRAPH:
                rows, ctx, last, mctx = self._repad
                part, nparts = plan_partitions(T, self.model.n_kv, mctx)
                kind, nt, nl = KIND_EAGER, T, T
            self.model.moe_capacity_tokens = t_max
            return kind, T, nt, nl, part, nparts, 0
        if b_max != bucket:
            rows, ctx, last, _ = self._repad
            self.meta.fill_decode(rows, ctx, last, pad_to=b_max)
            self.stats["ep_repadded_steps"] += 1
        return kind, b_max, b_max, b_max, part, nparts, b_max

    def _execute(self, kind, T, nt, nl, part, nparts, bucket, npt=0, greedy=0):
        if self._inject_device_us:  # fault injection: this step is slower on the device only
            torch.ops.mlop.device_delay(self._inject_device_us)
        if kind == KIND_GRAPH:
            graph, logits_buf = self.graphs[bucket]
            graph.replay()
            return self._gather(logits_buf, greedy)
        meta = self.meta.meta(T, nt, nl, part, nparts, npt)
        hidden = self.model.forward(self.meta.ids_d[:T], meta, self.kv)
        if nl == 0:
            return None
        return self._gather(self.model.logits_local(hidden[meta.logits_idx]), greedy)

    def _gather(self, local, greedy):
        """Vocab-parallel LM head -> what the sampler needs (CL3).  Greedy rows need only each
        rank's (max logit, its global index): an [n, 2] all-gather instead of the [n, V/TP]
        logits shard per rank (70B TP=8: 16 032 columns).  Ties keep the lowest vocabulary
        index, as an argmax over the full row does."""
        tp = self.model.ps.tp
        if tp.size == 1:
            return local
        if not greedy:
            return tp.all_gather(local, dim=-1)
        idx = ops.argmax(local) if local.is_cuda else local.argmax(-1)
        val = local.gather(1, idx.view(-1, 1)).float()
        pair = torch.cat([val, (idx.view(-1, 1) + self.model.vocab_start).float()], dim=1)  # [n, 2]
        allp = tp.all_gather(pair.contiguous(), dim=1).view(-1, tp.size, 2)  # [n, tp, 2]
        best = allp[:, :, 0].argmax(dim=1)  # first max: the lowest rank = the lowest vocab index
        return _Tokens(allp[torch.arange(allp.shape[0], device=allp.device), best, 1].to(torch.int64))

    def _sample(self, out, params, gen_index=None):
        return out.ids if isinstance(out, _Tokens) else self.sampler(out, params, gen_index)

    def _gen_index(self, rows, done_seqs):
        """Output position of each row's draw (seeded sampling): decode rows' generated count
        (it counts an in-flight token under async scheduling), then the prompts that completed."""
        return np.concatenate([self.r_gen[rows], np.asarray([len(s.output) for s in done_seqs], dtype=np.int64)])

    def worker_loop(self):
        """Non-zero TP ranks: replay rank 0's steps until it sends STOP."""
        assert self.step_sync is not None
        while True:
            hdr = self.step_sync.recv(self)
            if hdr[0] == KIND_STOP:
                return
            if hdr[0] == KIND_BARRIER:
                self._world_barrier()
                continue
            self._execute(*hdr)
            self._check_peers()
            self.stats["worker_steps"] += 1

    def sync_point(self):
        """Device sync + a barrier of the WHOLE world that the TP workers join too
        (they are parked in ``worker_loop``): the bench's timing brackets."""
        if self.step_sync is not None and self.step_sync.is_leader:
            self.step_sync.send(self, KIND_BARRIER, 0, 0, 0, 0, 0, 0)
        self._world_barrier()

    def _world_barrier(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        import torch.distributed as dist

        if dist.is_initialized():
            dist.barrier()
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)  # the barrier's own collective, on both sides

    def shutdown(self):
        if self.step_sync is not None and self.step_sync.is_leader:
            self.step_sync.send(self, KIND_STOP, 0, 0, 0, 0, 0, 0)

    # ----------------------------------------------------------- graphs --
    def capture_graphs(self):
        """Capture one decode graph per batch bucket (largest first, shared pool)."""
        m = self.model
        stream = torch.cuda.Stream(self.device)
        stream.wait_stream(torch.cuda.current_stream(self.device))
        self.graph_pool = torch.cuda.graph_pool_handle()
        empty = np.zeros(0, dtype=np.int32)
        t0 = time.perf_counter()
        verbose = False
        with torch.cuda.stream(stream):
            for bi, b in enumerate(sorted(self.buckets, reverse=True)):
                self.meta.fill_decode(empty, empty, np.zeros(0, dtype=np.int64), pad_to=b)
                self.meta.upload(b, b)
                m.moe_capacity_tokens = b  # EP: every rank's graph of bucket b exchanges b rows
                part, nparts = plan_partitions(b, m.n_kv, self.max_model_len)
                meta = self.meta.meta(b, b, b, part, nparts)
                ids = self.meta.ids_d[:b]
                # decode fills (fill_decode) give every row, padding included, its own logits row
                # in order: logits_idx is the identity, so the graph skips the row gather
                for _ in range(2 if bi == 0 else 1):  # warm-up (allocator, autotune, lazy init)
                    m.logits_local(m.forward(ids, meta, self.kv))
                stream.synchronize()
                if verbose:
                    print(f"[engine] capturing decode graph {bi + 1}/{len(self.buckets)} (batch {b}) "
                          f"at {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=self.graph_pool, stream=stream):
                    logits = m.logits_local(m.forward(ids, meta, self.kv))
                self.graphs[b] = (g, logits)
        torch.cuda.current_stream(self.device).wait_stream(stream)
        torch.cuda.synchronize(self.device)
        self.stats["graph_capture_ms"] = int(1e3 * (time.perf_counter() - t0))

    # ------------------------------------------------------ offline API --
    def generate(self, prompts, params: SamplingParams | list | None = None):
        """Offline batch API.  EP group: EVERY rank calls it (each with its own prompts, maybe
        none) and the ranks keep stepping together until the whole group is done."""
        if not isinstance(params, list):
            params = [params or SamplingParams()] * len(prompts)
        seqs = [self.add_request(p, sp) for p, sp in zip(prompts, params)]
        if self.ep_sync is not None:
            while True:
                self.step()
                if self.ep_sync.last_busy == 0 and all(s.status == Status.FINISHED for s in seqs):
                    return [s.output for s in seqs]
        while any(s.status != Status.FINISHED for s in seqs):
            self.step()
        return [s.output for s in seqs]
