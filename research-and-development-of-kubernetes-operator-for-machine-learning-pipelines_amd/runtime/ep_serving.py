"""Expert-parallel serving (config 5 at EP = N): one HTTP front over N data-parallel engines.

The engine's EP mode (``engine.EPSync``) makes every rank of a
DP-attention + EP group schedule its OWN requests while every MoE layer exchanges routed rows
with the other ranks (sync-free fixed-capacity all-to-all, ``parallel/moe.py``).  This module
puts that group behind ONE predictor endpoint, the way the operator deploys it: one pod, N
GPUs, ``python -m mlopamd.runtime.server --ep N`` (``server.launch_ranks`` starts one process
per GPU; rank 0 serves HTTP).

Per serving iteration, over the group's CPU (gloo) process group:

  1. rank 0 broadcasts ``{"stop", "new": [(rid, rank, prompt, params)]}`` -- the requests that
     arrived over HTTP since the last iteration, each assigned to the least-loaded rank;
  2. every rank admits its share and runs ONE ``engine.step()`` (the EP agreement inside lets a
     rank with nothing scheduled join the step's all-to-alls with a padding-only forward);
  3. ``all_gather_object`` of every rank's ``(rid, token, finished, reason)`` outputs and its
     running count; rank 0 completes the HTTP futures / stream queues and keeps the load table.

All ranks therefore call ``engine.step()`` the same number of times, in lock-step, which the
EP all-to-alls require.  An idle group keeps a heartbeat (one empty iteration per second) so
the gloo collectives never sit past their timeout.  Reference contract: one predictor per
model version behind the SeldonDeployment's endpoint (mlflow_operator.py:194-238).
"""
from __future__ import annotations

import itertools
import os
import threading
import time

from .backends import LLMBackend
from .sampler import SamplingParams


class _Out:
    __slots__ = ("seq_id", "token", "finished", "finish_reason")

    def __init__(self, rid, token, finished, reason):
        self.seq_id, self.token, self.finished, self.finish_reason = rid, token, finished, reason


def _params_dict(p: SamplingParams) -> dict:
    return {k: getattr(p, k) for k in p.__dataclass_fields__}


class EPGroupLoop:
    """The per-iteration protocol, shared by rank 0 (inside ``EPBackend``) and the other ranks."""

    def __init__(self, engine, ps):
        self.engine, self.ps = engine, ps
        self.group = ps.ep_cpu
        self.rank, self.world = ps.ep.rank, ps.ep.size
        self.local: dict[int, int] = {}  # local seq_id -> global request id
        self.iterations = 0

    def iterate(self, msg: dict | None) -> tuple[dict, list]:
        """One lock-step iteration.  ``msg`` is rank 0's broadcast (None elsewhere).  Returns
        (the broadcast message, every rank's [(outputs, running)])."""
        import torch.distributed as dist

        box = [msg]
        dist.broadcast_object_list(box, src=dist.get_global_rank(self.group, 0), group=self.group)
        msg = box[0]
        for rid, r, prompt, pd in msg["new"]:
            if r == self.rank:
                seq = self.engine.add_request(prompt, SamplingParams(**pd))
                self.local[seq.seq_id] = rid
        outs = []
        if not msg["stop"]:
            for o in self.engine.step():
                rid = self.local.get(o.seq_id)
                if rid is None:
                    continue
                outs.append((rid, int(o.token), bool(o.finished), o.finish_reason))
                if o.finished:
                    self.local.pop(o.seq_id, None)
        gathered = [None] * self.world
        dist.all_gather_object(gathered, (outs, self.engine.num_running + len(self.engine.waiting)), group=self.group)
        self.iterations += 1
        return msg, gathered

    def worker(self):
        """Ranks > 0: follow rank 0's iterations until it broadcasts stop."""
        while True:
            msg, _ = self.iterate(None)
            if msg["stop"]:
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
        self.heartbeat_s = float(os.environ.get("MLOP_EP_HEARTBEAT_S", 1.0))
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
            new = []
            for r in pend:
                rid = next(self._rid)
                self._by_rid[rid] = r
                new.append((rid, self._assign(), list(r.prompt), _params_dict(r.params)))
            msg, gathered = self.group_loop.iterate({"stop": stop, "new": new})
            last = time.perf_counter()
            if stop:
                break
            self.steps += 1
            now = time.perf_counter()
            n_tok = 0
            busy = False
            for rank, (outs, running) in enumerate(gathered):
                self.load[rank] = running
                busy = busy or running > 0
                for rid, tok, fin, reason in outs:
                    n_tok += 1
                    self._deliver(_Out(rid, tok, fin, reason), now)
            if self.metrics:
                self.metrics.engine_steps.labels(**self.metrics.labels).inc()
                if n_tok:
                    self.metrics.engine_tokens.labels(**self.metrics.labels).inc(n_tok)
                m = self.metrics
                m.running.labels(**m.labels).set(sum(self.load))
        self.stopped.set()

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
