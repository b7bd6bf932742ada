"""Expert-parallel serving (config 5 at EP = N): one HTTP front over N data-parallel engines.

The engine's EP mode (``engine.EPSync``) makes every rank of a
DP-attention + EP group schedule its OWN requests while every MoE layer exchanges routed rows
with the other ranks (sync-free fixed-capacity all-to-all, ``parallel/moe.py``).  This module
puts that group behind ONE predictor endpoint, the way the operator deploys it: one pod, N
GPUs, ``python -m mlopamd.runtime.server --ep N`` (``server.launch_ranks`` starts one process
per GPU; rank 0 serves HTTP).

Per serving iteration, over the group's host all-gather (parallel/comm.py ``HostAllGather``: one
POSIX shared-memory hop per exchange, ops/csrc/shm_allgather.cc; gloo only when shared memory is
unavailable), with fixed-layout int64 words (no pickles: a peer's message can only ever be
numbers):

  1. exchange 1 (a broadcast: only rank 0's words are read): [stop, n_new, request records]
     (``_pack``): request id, assigned rank (the least-loaded), prompt, sampling parameters
     (floats as their bit patterns).  Requests are validated on rank 0 BEFORE they are sent
     (``Engine.check_request``): a bad one fails its own HTTP future and never reaches a rank.
     At most one slot of records travels per iteration; the rest wait for the next one;
  2. every rank admits its share (an admission that still fails is reported back, below) and
     runs ONE ``engine.step()`` (the EP agreement inside -- ``EPSync``, the same kind of
     exchange -- lets a rank with nothing scheduled join the step's expert exchange with a
     padding-only forward);
  3. exchange 2 (an all-gather): [n_out, running, rows of (request id, token, finished, reason
     code)] from every rank; rank 0 completes the HTTP futures / stream queues, fails the
     requests a rank could not admit, and keeps the load table.

All ranks therefore call ``engine.step()`` the same number of times, in lock-step, which the
EP exchange requires.  An idle group keeps a heartbeat (one empty iteration per second) so a
dead rank is noticed (every exchange has a deadline).  Reference contract: one predictor per
model version behind the SeldonDeployment's endpoint (mlflow_operator.py:194-238).
"""
from __future__ import annotations

import itertools
import os
import threading
import time

import numpy as np
import torch

from .backends import LLMBackend, _set_exc
from .sampler import SamplingParams

REASONS = {None: 0, "stop": 1, "length": 2, "abort": 3}
REASON_NAMES = {v: k for k, v in REASONS.items()}
FAILED = -1  # reason code of a request a rank could not admit


class _Out:
    __slots__ = ("seq_id", "token", "finished", "finish_reason")

    def __init__(self, rid, token, finished, reason):
        self.seq_id, self.token, self.finished, self.finish_reason = rid, token, finished, reason


def _f2i(x: float) -> int:
    return int(np.array([x], dtype=np.float64).view(np.int64)[0])


def _i2f(i: int) -> float:
    return float(np.array([i], dtype=np.int64).view(np.float64)[0])


def packed_words(prompt, params) -> int:
    """int64 words one request record takes in ``_pack``."""
    return 11 + len(params.stop_token_ids) + len(prompt)


def _pack(new) -> torch.Tensor:
    """[(rid, rank, prompt, SamplingParams)] -> one int64 tensor of records:
    rid, rank, len(prompt), max_tokens, top_k, ignore_eos, len(stop), has_seed, seed,
    temperature bits, top_p bits, *stop_token_ids, *prompt."""
    out = []
    for rid, r, prompt, p in new:
        stop = list(p.stop_token_ids)
        out += [rid, r, len(prompt), int(p.max_tokens), int(p.top_k), int(bool(p.ignore_eos)), len(stop),
                int(p.seed is not None), int(p.seed or 0), _f2i(p.temperature), _f2i(p.top_p), *stop, *prompt]
    return torch.tensor(out, dtype=torch.int64)


def _unpack(buf: torch.Tensor, n: int):
    v = buf.tolist()
    i, out = 0, []
    for _ in range(n):
        rid, r, plen, mt, tk, ign, nstop, hs, seed, tb, pb = v[i:i + 11]
        i += 11
        stop = v[i:i + nstop]
        i += nstop
        prompt = v[i:i + plen]
        i += plen
        out.append((rid, r, prompt, SamplingParams(max_tokens=mt, temperature=_i2f(tb), top_k=tk, top_p=_i2f(pb),
                                                   ignore_eos=bool(ign), stop_token_ids=stop,
                                                   seed=seed if hs else None)))
    return out


class EPGroupLoop:
    """The per-iteration protocol, shared by rank 0 (inside ``EPBackend``) and the other ranks."""

    def __init__(self, engine, ps):
        from ..parallel.comm import make_host_allgather

        self.engine, self.ps = engine, ps
        self.group = ps.ep_cpu
        self.rank, self.world = ps.ep.rank, ps.ep.size
        self.local: dict[int, int] = {}  # local seq_id -> global request id
        self.iterations = 0
        # one slot holds a longest prompt's record, and every output row of a full engine
        # one slot must hold the largest request any backend accepts (packed_words: a prompt of
        # max_model_len ids + MAX_STOP_IDS stop ids + the header) and a step's output records
        from .sampler import MAX_STOP_IDS

        self.max_words = max(32768, engine.max_model_len + MAX_STOP_IDS + 64, 8 * engine.cfg.max_num_seqs + 64)
        self.xg = make_host_allgather(self.group, self.max_words)
        self._none = torch.zeros(0, dtype=torch.int64)

    def iterate(self, stop: bool = False, new=()) -> tuple[bool, list]:
        """One lock-step iteration.  ``stop`` / ``new`` [(rid, rank, prompt, params)]: rank 0's
        (ignored elsewhere; their packed records must fit one slot).  Returns (stop, every
        rank's (outputs [n, 4] int64, running))."""
        if self.rank == 0:
            head = torch.tensor([int(stop), len(new)], dtype=torch.int64)
            msg = torch.cat([head, _pack(new)]) if new else head
        else:
            msg = self._none
        w = self.xg.exchange(msg)[0]  # rank 0's words
        stop, n_new = int(w[0]), int(w[1])
        new = _unpack(w[2:], n_new) if n_new else ()
        rows, failed = [], []
        for rid, r, prompt, params in new:
            if r != self.rank:
                continue
            try:
                seq = self.engine.add_request(prompt, params)
                self.local[seq.seq_id] = rid
            except Exception:  # noqa: BLE001 - reported to rank 0, which fails that request only
                failed.append(rid)
        if not stop:
            for o in self.engine.step():
                rid = self.local.get(o.seq_id)
                if rid is None:
                    continue
                rows.append((rid, int(o.token), int(bool(o.finished)), REASONS.get(o.finish_reason, 0)))
                if o.finished:
                    self.local.pop(o.seq_id, None)
        rows += [(rid, 0, 1, FAILED) for rid in failed]
        running = self.engine.num_running + len(self.engine.waiting)
        msg = torch.tensor([len(rows), running] + [v for row in rows for v in row], dtype=torch.int64)
        parts = self.xg.exchange(msg)
        # copies: the exchange's buffer is reused by the next iteration
        gathered = [(p[2:2 + 4 * int(p[0])].reshape(-1, 4).clone(), int(p[1])) for p in parts]
        self.iterations += 1
        return bool(stop), gathered

    def worker(self):
        """Ranks > 0: follow rank 0's iterations until it sends stop."""
        while True:
            stop, _ = self.iterate()
            if stop:
                return


class EPBackend(LLMBackend):
    """Rank 0's serving backend: the V2 server's LLM backend whose engine loop drives the whole
    EP group (``EPGroupLoop``) instead of one local engine."""

    def __init__(self, engine, ps, metrics=None, tokenizer=None, name: str = "model"):
        super().__init__(engine, metrics, tokenizer=tokenizer, name=name)
        self.group_loop = EPGroupLoop(engine, ps)
        self.load = [0] * ps.ep.size
        self._rid = itertools.count()
        self._by_rid: dict[int, object] = {}
        self.heartbeat_s = 1.0  # an idle group's empty iteration per second: a dead rank is noticed
        self.stopped = threading.Event()

    def _assign(self) -> int:
        r = min(range(len(self.load)), key=lambda i: (self.load[i], i))
        self.load[r] += 1
        return r

    def _loop(self):
        last = time.perf_counter()
        busy = False
        while True:
            with self._lock:
                pend, self._pending = self._pending, []
            stop = self._stop
            if not pend and not busy and not stop:
                # idle group: wait for a request, but iterate at least once per heartbeat
                self._wake.wait(min(0.05, self.heartbeat_s))
                self._wake.clear()
                if time.perf_counter() - last < self.heartbeat_s and not self._pending and not self._stop:
                    continue
                with self._lock:
                    pend, self._pending = self._pending, []
                stop = self._stop
            new, room = [], self.group_loop.max_words - 2
            for i, r in enumerate(pend):
                try:  # validated HERE, before any rank sees it: a bad request fails alone
                    self.engine.check_request(list(r.prompt), r.params)
                    if packed_words(r.prompt, r.params) > self.group_loop.max_words - 2:
                        raise ValueError("request too large for the expert-parallel group's control slot")
                except Exception as e:  # noqa: BLE001
                    r.loop.call_soon_threadsafe(_set_exc, r.future, e)
                    continue
                need = packed_words(r.prompt, r.params)
                if need > room:  # one slot per iteration: the rest go next iteration, in order
                    with self._lock:
                        self._pending[:0] = pend[i:]
                    break
                room -= need
                rid = next(self._rid)
                self._by_rid[rid] = r
                new.append((rid, self._assign(), list(r.prompt), r.params))
            stop_now, gathered = self.group_loop.iterate(stop, new)
            last = time.perf_counter()
            if stop_now:
                break
            self.steps += 1
            now = time.perf_counter()
            n_tok = 0
            busy = False
            for rank, (outs, running) in enumerate(gathered):
                self.load[rank] = running
                busy = busy or running > 0
                for rid, tok, fin, code in outs.tolist():
                    if code == FAILED:
                        self._fail(rid, RuntimeError(f"request {rid} could not be admitted on rank {rank}"))
                        continue
                    n_tok += 1
                    self._deliver(_Out(rid, tok, bool(fin), REASON_NAMES.get(code)), now)
            if self.metrics:
                self.metrics.mark_step(n_tok, time.perf_counter())
                m = self.metrics
                m.running.labels(**m.labels).set(sum(self.load))
        self.stopped.set()

    def _fail(self, rid, exc):
        r = self._by_rid.pop(rid, None)
        if r is not None:
            if r.queue is not None:
                r.loop.call_soon_threadsafe(r.queue.put_nowait, None)
            r.loop.call_soon_threadsafe(_set_exc, r.future, exc)

    def _deliver(self, o, now):
        r = self._by_rid.get(o.seq_id)
        if r is None:
            return
        if r.t_first is None:
            r.t_first = now
            if self.metrics:
                self.metrics.ttft.labels(**self.metrics.labels).observe(now - r.t0)
                self.metrics.tokens_in.labels(**self.metrics.labels).inc(len(r.prompt))
        r.tokens.append(o.token)
        if r.queue is not None:
            r.loop.call_soon_threadsafe(r.queue.put_nowait, o.token)
        if o.finished:
            self._by_rid.pop(o.seq_id, None)
            res = {"output_ids": list(r.tokens), "finish_reason": o.finish_reason,
                   "ttft": r.t_first - r.t0, "latency": now - r.t0, "prompt_tokens": len(r.prompt)}
            if self.metrics:
                m = self.metrics
                m.tokens_out.labels(**m.labels).inc(len(r.tokens))
                if len(r.tokens) > 1:
                    m.tpot.labels(**m.labels).observe((now - r.t_first) / (len(r.tokens) - 1))
            if r.queue is not None:
                r.loop.call_soon_threadsafe(r.queue.put_nowait, None)
            from .backends import _set_res

            r.loop.call_soon_threadsafe(_set_res, r.future, res)


def serve_ep(args, metrics):
    """Entry from ``runtime.server.main`` for ``--ep N`` (one call per rank)."""
    import torch
    from aiohttp import web

    from .backends import load_tokenizer
    from .server import engine_kwargs_from_env, make_app
    from .tp_worker import build_tp_engine

    ep = int(os.environ.get("WORLD_SIZE", args.ep))
    rank = int(os.environ.get("RANK", 0))
    if rank == 0 and os.environ.get("MLOP_INJECT_START_ERROR"):
        raise RuntimeError(os.environ["MLOP_INJECT_START_ERROR"])
    device = "cpu" if (args.device == "cpu" or not torch.cuda.is_available()) else None
    eng, ps = build_tp_engine(args.architecture or "mixtral-8x7b", 1, device=device, ep=ep,
                              engine_kwargs=engine_kwargs_from_env(), model_uri=args.model_uri,
                              seed=int(os.environ.get("MLOP_SEED", 0)))
    if eng.ep_sync is None:
        raise SystemExit(f"--ep {ep}: {args.architecture} is not a MoE model (no expert-parallel mode)")
    if ps.ep.rank != 0:
        EPGroupLoop(eng, ps).worker()
        return
    backend = EPBackend(eng, ps, metrics, tokenizer=load_tokenizer(eng.checkpoint_dir), name=args.name).start()
    try:
        web.run_app(make_app(backend, metrics, version=args.version), host=args.host, port=args.port, print=None)
    finally:
        backend.stop()
