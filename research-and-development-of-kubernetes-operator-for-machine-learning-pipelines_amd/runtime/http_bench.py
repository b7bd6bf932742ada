"""The headline load driven end to end through the serving stack (``bench.py --http``).

What ``bench.py`` measures by default is the engine's served rate with requests handed to
``Engine.add_request`` in-process.  This mode puts every layer of the deployed path in the
loop (reference serving path: the SeldonDeployment's ``protocol:
kfserving`` endpoint, mlflow_operator.py:225-238):

  1. registry -> MlflowModel CR -> operator -> SeldonDeployment -> the local Seldon stand-in
     starts the predictor CONTAINER COMMAND as a fresh OS process (``ProcessLauncher``) on
     this node's GPU: CR -> ready therefore includes process start, ``import torch``, HIP
     init, weight init, KV pool and graph capture (``p50_cr_ready_process_s``);
  2. ``--batch`` closed-loop HTTP clients (aiohttp) post V2 ``/v2/models/{m}/generate``
     requests through the weighted ``Router`` (the Istio stand-in), first cohort at
     staggered output lengths like the engine-direct bench;
  3. the predictor exports ``mlop_engine_steps_total`` / ``mlop_engine_tokens_total``; after
     ``warmup`` engine steps the window opens, and it closes after ``steps`` more: value =
     generated tokens in the window / its wall time.
"""
from __future__ import annotations

import asyncio
import re
import time

import numpy as np

_NS, _NAME = "serving", "llm"


async def _scrape(session, url) -> dict:
    async with session.get(url) as r:
        txt = await r.text()
    out = {}
    for name in ("mlop_engine_steps_total", "mlop_engine_tokens_total", "mlop_prompt_tokens_total",
                 "mlop_num_requests_waiting", "mlop_num_requests_running", "mlop_engine_clock_seconds",
                 "mlop_engine_tokens_at_clock"):
        m = re.search(rf"^{name}\{{[^}}]*\}} ([0-9.e+]+)$", txt, re.M)
        out[name] = float(m.group(1)) if m else 0.0
    return out


async def _start_stack(model: str, batch: int, engine_env: dict | None, ready_timeout_s: float, gpus=None):
    """registry + operator + the local Seldon stand-in with a ProcessLauncher (fresh predictor
    processes) + the weighted Router.  ``gpus``: device indices the launcher may hand out
    (default: every visible GPU)."""
    from ..controller.app import make_operator
    from ..controller.clock import RealClock
    from ..controller.crd import OperatorSettings
    from ..controller.kube import FakeKube
    from ..controller.local import FakeSeldonController, GpuPool, ProcessLauncher, Router
    from ..controller.mlflow import LocalMlflowClient, SqliteRegistry
    from ..controller.prometheus import LocalProm, MetricStore

    kube, reg = FakeKube(), SqliteRegistry()
    reg.create_model_version(_NAME, f"mlflow-artifacts:/1/{model}/artifacts/model",
                             tags={"mlop.architecture": model, "mlop.runtime": "mlop-llm"})
    reg.set_alias(_NAME, "champion", 1)
    op, _ = make_operator(kube, LocalMlflowClient(reg), LocalProm(MetricStore()), RealClock(), OperatorSettings())
    env = {"MLOP_ENGINE_MAX_NUM_SEQS": str(batch), "MLOP_KERNEL_SAMPLE_S": "0"}
    env.update(engine_env or {})
    pool = GpuPool(gpus) if gpus is not None else GpuPool.detect()
    launcher = ProcessLauncher(extra_env=env, gpus=pool if pool.devices else None, ready_timeout_s=ready_timeout_s)
    ctl = FakeSeldonController(kube, launcher, RealClock()).start()
    await op.start()
    return kube, op, ctl, Router(ctl)


async def _create_and_wait_ready(kube, ctl, batch: int, ready_timeout_s: float) -> dict:
    """MlflowModel CR -> ... -> the predictor process answers /v2/health/ready and the CR
    reports ready; the clock runs from the CR create."""
    from ..controller.crd import GROUP, PLURAL, VERSION
    from ..controller.local import mlflow_model_cr, wait_for

    t0 = time.perf_counter()
    await kube.create(GROUP, VERSION, _NS, PLURAL, mlflow_model_cr(_NAME, _NS, _NAME, "champion",
                                                                   maxNumSeqs=batch, maxModelLen=1024))

    async def ready():
        o = await kube.get(GROUP, VERSION, _NS, PLURAL, _NAME)
        for p in ctl.pods.values():  # a predictor that cannot start fails the run now
            if "error" in p.extra:
                raise RuntimeError(f"predictor {p.predictor} failed to start: {p.extra['error']}")
        return (o.get("status") or {}).get("ready") == "True"

    await wait_for(ready, ready_timeout_s, poll_s=0.01)
    cr_ready = time.perf_counter() - t0
    pod = next(iter(ctl.pods.values()))
    return {"cr_ready_process_s": round(cr_ready, 3), "predictor_process_ready_s": round(pod.extra.get("ready_s", 0.0), 3),
            # CR create -> the launcher's spawn (operator reconcile, SeldonDeployment, GPU grant)
            "predictor_spawn_s": round(pod.extra.get("t_start", t0) - t0, 3),
            "predictor_gpus": pod.extra.get("gpus"), "pod": pod}


async def cr_ready_process(model: str = "llama3-8b", batch: int = 2048, engine_env: dict | None = None,
                           samples: int = 1, gpus=None, ready_timeout_s: float = 900.0) -> dict:
    """CR -> ready with the predictor as a FRESH OS process (process start, imports, HIP init,
    weights, KV pool, graph capture all inside), ``samples`` times on a fresh stack each; the
    predictor is torn down again.  The default ``bench.py`` line reports its median as
    ``p50_cr_ready_s``."""
    vals, last = [], {}
    for _ in range(max(1, samples)):
        kube, op, ctl, _router = await _start_stack(model, batch, engine_env, ready_timeout_s, gpus)
        try:
            last = await _create_and_wait_ready(kube, ctl, batch, ready_timeout_s)
            vals.append(last["cr_ready_process_s"])
            try:  # the predictor's own start-up phases (runtime/server.py STARTUP)
                import aiohttp

                async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=5)) as s:
                    async with s.get(last["pod"].endpoint + "/v2/debug/startup") as r:
                        last["predictor_startup"] = await r.json()
            except Exception:  # noqa: BLE001
                pass
        finally:
            await ctl.stop()
            await op.stop()
    vals.sort()
    n = len(vals)
    p50 = vals[n // 2] if n % 2 else 0.5 * (vals[n // 2 - 1] + vals[n // 2])
    return {"p50_cr_ready_process_s": round(p50, 3), "cr_ready_process_samples_s": vals,
            "predictor_spawn_s": last.get("predictor_spawn_s"),
            "predictor_process_ready_s": last.get("predictor_process_ready_s"),
            "predictor_gpus": last.get("predictor_gpus"), "predictor_startup": last.get("predictor_startup")}


async def run(model: str = "llama3-8b", batch: int = 2048, prompt_len: int = 256, output_len: int = 256,
              steps: int = 20, warmup: int = 5, engine_env: dict | None = None, ready_timeout_s: float = 900.0,
              ramp_timeout_s: float = 600.0, gpus=None) -> dict:
    import aiohttp

    from ..models.config import get_config

    ns, name = _NS, _NAME
    kube, op, ctl, router = await _start_stack(model, batch, engine_env, ready_timeout_s, gpus)
    out: dict = {"mode": "http", "path": "operator + ProcessLauncher + V2 HTTP + Router"}
    try:
        r = await _create_and_wait_ready(kube, ctl, batch, ready_timeout_s)
        pod = r.pop("pod")
        out["p50_cr_ready_process_s"] = r["cr_ready_process_s"]
        out["predictor_process_ready_s"] = r["predictor_process_ready_s"]
        out["predictor_gpus"] = r["predictor_gpus"]
        metrics_url = pod.endpoint + "/metrics"
        V = get_config(model).vocab_size
        rng = np.random.default_rng(1234)
        lo = min(1000, V // 4)
        stop = asyncio.Event()
        stats = {"requests": 0, "errors": 0}

        async def client(session, i):
            first = 1 + (i * output_len) // batch  # staggered first cohort (steady-state age mix)
            mt = first
            while not stop.is_set():
                ids = rng.integers(lo, V - lo, size=prompt_len).tolist()
                payload = {"input_ids": ids, "parameters": {"max_tokens": int(mt), "ignore_eos": True}}
                code, _, _ = await router.post(ns, name, f"/v2/models/{name}/generate", payload, session)
                stats["requests"] += 1
                if code != 200:
                    stats["errors"] += 1
                    await asyncio.sleep(0.05)
                mt = output_len

        conn = aiohttp.TCPConnector(limit=0)
        async with aiohttp.ClientSession(connector=conn, timeout=aiohttp.ClientTimeout(total=None)) as session:
            tasks = [asyncio.get_running_loop().create_task(client(session, i)) for i in range(batch)]
            # ramp (as the engine-direct bench): the first cohort's prompts are all prefilled and
            # the admission queue is down to ~2 steps of arrivals.  Scrapes are sparse (every
            # 0.25 s in the ramp, 0.1 s in the window): the exposition runs on the predictor's
            # event loop and a tight poll would take host time from its engine thread.
            backlog = max(8, 2 * batch // max(1, output_len))
            t_ramp = time.perf_counter()
            while time.perf_counter() - t_ramp < ramp_timeout_s:
                cur = await _scrape(session, metrics_url)
                if (cur["mlop_prompt_tokens_total"] >= batch * prompt_len
                        and cur["mlop_num_requests_waiting"] <= backlog):
                    break
                if int(4 * (time.perf_counter() - t_ramp)) % 40 == 0:  # a progress line every ~10 s
                    print(f"[http_bench] ramp {time.perf_counter() - t_ramp:.0f}s running="
                          f"{cur['mlop_num_requests_running']:.0f} waiting={cur['mlop_num_requests_waiting']:.0f} "
                          f"prompt_tokens={cur['mlop_prompt_tokens_total']:.0f}", flush=True)
                await asyncio.sleep(0.25)
            out["http_ramp_s"] = round(time.perf_counter() - t_ramp, 2)
            s_ramp = cur
            while True:  # warmup steps
                cur = await _scrape(session, metrics_url)
                if cur["mlop_engine_steps_total"] >= s_ramp["mlop_engine_steps_total"] + warmup:
                    break
                await asyncio.sleep(0.1)
            t_a, a = time.perf_counter(), cur
            while True:  # the timed steps (window = whole scrape intervals, >= steps engine steps)
                await asyncio.sleep(0.1)
                cur = await _scrape(session, metrics_url)
                if cur["mlop_engine_steps_total"] >= a["mlop_engine_steps_total"] + steps:
                    break
            t_b, b = time.perf_counter(), cur
            stop.set()
            for t in tasks:
                t.cancel()
            await asyncio.gather(*tasks, return_exceptions=True)
        n_steps = b["mlop_engine_steps_total"] - a["mlop_engine_steps_total"]
        # the window's time on the predictor's engine clock (end of the first / last counted
        # step), not between the two scrape responses: a scrape answered late by the busy event
        # loop lengthened the client-side window by up to ~12 % (two 33.7k vs 38.5k samples).
        # Tokens from the SAME snapshot as each clock reading (metrics.mark_step)
        ck = b["mlop_engine_clock_seconds"] - a["mlop_engine_clock_seconds"]
        if a["mlop_engine_clock_seconds"] > 0 and ck > 0:
            dt = ck
            toks = b["mlop_engine_tokens_at_clock"] - a["mlop_engine_tokens_at_clock"]
        else:
            dt = t_b - t_a
            toks = b["mlop_engine_tokens_total"] - a["mlop_engine_tokens_total"]
        out.update(served_tokens_per_sec_http=round(toks / dt, 2), http_window_steps=int(n_steps),
                   http_ms_per_step=round(1e3 * dt / max(n_steps, 1), 3),
                   http_window_client_s=round(t_b - t_a, 3), http_window_engine_s=round(ck, 3),
                   http_requests=stats["requests"], http_errors=stats["errors"],
                   http_running_at_end=int(b["mlop_num_requests_running"]))
    finally:
        await ctl.stop()
        await op.stop()
    return out


def main(a, steps: int | None = None, warmup: int | None = None, gpus=None, extra_env: dict | None = None) -> dict:
    env = {"MLOP_ENGINE_MAX_NUM_BATCHED_TOKENS": str(a.max_batched_tokens),
           "MLOP_ENGINE_MAX_MODEL_LEN": str(a.max_model_len),
           "MLOP_ENGINE_PREFILL_MIN_BATCH": str(a.prefill_min_batch),
           "MLOP_ENGINE_MAX_DECODE_GAP": str(a.max_decode_gap)}
    env.update(extra_env or {})
    return asyncio.run(run(a.model, a.batch, a.prompt_len, a.output_len, a.steps if steps is None else steps,
                           a.warmup if warmup is None else warmup, gpus=gpus, engine_env=env))
