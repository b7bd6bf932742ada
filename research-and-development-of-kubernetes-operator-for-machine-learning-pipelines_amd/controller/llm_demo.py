"""BASELINE configs 2, 3 and 5 end to end on ONE MI355X box (no cluster, no network).

  registry (sqlite MLflow over REST) --alias--> MlflowModel CR --> operator
  --> SeldonDeployment (mlop-llm predictors, HBM placement annotations)
  --> fake Seldon controller starts REAL runtime server processes on the GPU
      (random-init Llama / Mixtral, HIP kernels, hipGraph decode)
  --> weighted router sends /generate load --> Scraper feeds the local
      Prometheus from every pod's /metrics (Seldon executor series + TPOT +
      amd-smi gauges) --> canary gate (reference thresholds + GPU guards)
  --> promotion to 100 % or automatic rollback.

Every predictor here is an OS process on the same GPU (two 8B models = 32 GB,
two Mixtral-8x7B = 187 GB: both fit one 288 GB MI355X), which is how one box
stands in for the two 1-GPU pods of config 3.  ``regress`` injects a fault into
the NEW version's pods only (per-predictor env of the launcher): ``latency``
(+ s per request), ``errors`` (HTTP 500 share), ``tpot`` (a device delay kernel in every
engine step: slower on the GPU only, with the latency thresholds loosened so that only the
GPU-side TPOT guard can decide) — the gate must roll it back.
"""
from __future__ import annotations

import asyncio
import tempfile
import time
from pathlib import Path

import numpy as np

FAULTS = {
    None: {},
    "latency": {"MLOP_INJECT_LATENCY_S": "0.25"},
    "errors": {"MLOP_INJECT_ERROR_RATE": "0.3"},
    # device-only slowdown: every engine step of v2 also runs a device delay kernel, while the
    # HTTP layer is untouched; the gate's latency thresholds are loosened for this case (GATES)
    # so only the GPU-side TPOT guard can reject it.  The delay scales with the model
    # (_fault_env): 0.2 ms on the tiny shapes (a tiny-llama step is ~0.16 ms: TPOT x ~2; 1.5 ms
    # made p95 / mean 10x worse than v1, beyond any loosened latency bound), 2 ms at real size
    # (an 8B decode step at concurrency 16 is ~4.9 ms: 0.2 ms gave TPOT x 1.04-1.11 and the
    # canary promoted)
    "tpot": {"MLOP_INJECT_STEP_DEVICE_US": "200"},
}


def _fault_env(regress: str | None, arch: str) -> dict:
    env = dict(FAULTS[regress])
    if regress == "tpot":
        from ..models.config import get_config

        env["MLOP_INJECT_STEP_DEVICE_US"] = "200" if get_config(arch).hidden_size <= 1024 else "2000"
    return env

# per-regression gate overrides: "tpot" keeps the TPOT guard at its 1.10 default and lets p95 /
# mean latency rise 10x, i.e. the Seldon-executor latency gate alone would promote v2
GATES = {
    "tpot": {"thresholds": {"latency_95th": 9.0, "latency_avg": 9.0}, "gpuGuards": {"tpot_avg": 1.10}},
}


async def run_llm_canary(arch: str = "tiny-llama", regress: str | None = None, device: str = "cuda",
                         namespace: str = "llm", concurrency: int = 8, prompt_len: int = 32,
                         max_tokens: int = 16, warm_requests: int = 16, timeout_s: float = 600.0,
                         engine_env: dict | None = None, gpu_slots: int | None = None) -> dict:
    import aiohttp

    from .app import OperatorMetrics, make_operator
    from .clock import RealClock
    from .crd import GROUP, PLURAL, SELDON_GROUP, SELDON_PLURAL, SELDON_VERSION, VERSION, OperatorSettings
    from .kube import FakeKube
    from .local import FakeSeldonController, GpuPool, ProcessLauncher, Router, mlflow_model_cr, wait_for
    from .mlflow import MlflowRestClient, SqliteRegistry, serve_registry
    from .prometheus import MetricStore, PromClient, Scraper, serve_prometheus
    from ..models.config import get_config

    t_start = time.perf_counter()
    tmp = Path(tempfile.mkdtemp(prefix="mlop-llm-demo-"))
    name = "llm"
    tags = {"mlop.runtime": "mlop-llm", "mlop.architecture": arch}
    reg = SqliteRegistry(str(tmp / "mlflow.db"))
    reg_runner, reg_url = await serve_registry(reg)
    mlflow = MlflowRestClient(reg_url)
    await mlflow.create_registered_model(name)
    await mlflow.create_model_version(name, f"mlflow-artifacts:/1/{arch}-v1/artifacts/model", tags=tags)
    await mlflow.set_alias(name, "champion", 1)

    clock = RealClock()
    store = MetricStore()
    scraper = Scraper(store, clock, interval_s=0.5)
    prom_runner, prom_url = await serve_prometheus(store)
    kube = FakeKube()
    prom = PromClient(prom_url)
    op, rec = make_operator(kube, mlflow, prom, clock, OperatorSettings(), metrics=OperatorMetrics())
    env = {"MLOP_DEVICE": device, "MLOP_ENGINE_MAX_NUM_SEQS": str(max(16, 2 * concurrency)),
           "MLOP_ENGINE_MAX_MODEL_LEN": "1024", "MLOP_ENGINE_MAX_NUM_BATCHED_TOKENS": "2048"}
    env.update(engine_env or {})
    pool = GpuPool.detect()
    if device == "cpu":
        pool = GpuPool(8)
    # one predictor per GPU when the node has a GPU per canary pod (config 3); a 1-GPU box
    # time-shares its card between the two versions (both fit 288 GB)
    slots = gpu_slots or (1 if len(pool.devices) >= 2 else 2)
    pool.slots = slots
    launcher = ProcessLauncher(scraper, extra_env=env, per_predictor_env={"v2": _fault_env(regress, arch)}, gpus=pool)
    ctl = FakeSeldonController(kube, launcher, clock).start()
    router = Router(ctl)
    scraper.start()
    await op.start()
    canary = {"step": 30, "intervalSeconds": 3, "attemptDelaySeconds": 1,
              "maxAttempts": 6, "windowSeconds": 8, "errorRateFloor": 0.01,
              "latencyFloorSeconds": 0.02,
              # shared-GPU pods: power / HBM of the card are common to both
              "gpuGuards": {"tpot_avg": 1.5}}
    canary.update(GATES.get(regress, {}))
    cr = mlflow_model_cr(name, namespace, name, "champion", interval=2, canary=canary,
                         maxNumSeqs=max(16, 2 * concurrency), maxModelLen=1024)
    t_cr = time.perf_counter()
    await kube.create(GROUP, VERSION, namespace, PLURAL, cr)

    last_log = [0.0]

    async def cr_status():
        st = (await kube.get(GROUP, VERSION, namespace, PLURAL, name)).get("status") or {}
        for p in ctl.pods.values():  # a predictor process that cannot start ends the demo now
            if "error" in p.extra and p.predictor == "v1":
                raise RuntimeError(f"predictor {p.predictor} failed to start: {p.extra['error']}")
        now = time.perf_counter()
        if now - last_log[0] > 10:  # progress line (long real-size starts print nothing else)
            last_log[0] = now
            print(f"[llm_demo {now - t_start:7.1f}s] phase={st.get('phase')} ready={st.get('ready')} "
                  f"pods={sorted(p.predictor for p in ctl.pods.values())}", flush=True)
        return st

    async def is_ready():
        return (await cr_status()).get("ready") == "True"

    await wait_for(is_ready, timeout_s=timeout_s)
    cr_ready_s = time.perf_counter() - t_cr
    V = get_config(arch).vocab_size
    rng = np.random.default_rng(0)
    served = {"n": 0, "errors": 0, "tokens": 0, "by_predictor": {}}
    stop = asyncio.Event()

    async def worker(session, limit):
        i = 0
        while not stop.is_set() and (limit is None or i < limit):
            ids = rng.integers(2, V - 2, size=prompt_len).tolist()
            payload = {"input_ids": ids, "parameters": {"max_tokens": max_tokens, "ignore_eos": True}}
            code, body, pred = await router.post(namespace, name, f"/v2/models/{name}/generate", payload, session)
            if code == 200:
                served["n"] += 1
                served["tokens"] += len(body["output_ids"])
                served["by_predictor"][pred] = served["by_predictor"].get(pred, 0) + 1
            else:
                served["errors"] += 1
            i += 1

    out = {"config": f"{arch} / mlop-llm / {device}", "cr_ready_s": round(cr_ready_s, 3),
           "predictor_gpus": {p.predictor: p.extra.get("gpus") for p in ctl.pods.values()},
           "predictor_process_ready_s": {p.predictor: round(p.extra.get("ready_s", 0.0), 3)
                                         for p in ctl.pods.values()}}
    async with aiohttp.ClientSession() as session:
        t0 = time.perf_counter()
        await asyncio.gather(*(worker(session, max(1, warm_requests // concurrency)) for _ in range(concurrency)))
        dt = time.perf_counter() - t0
        out["warm_tokens_per_s"] = round(served["tokens"] / dt, 1)
        bg = [asyncio.get_running_loop().create_task(worker(session, None)) for _ in range(concurrency)]
        await mlflow.create_model_version(name, f"mlflow-artifacts:/1/{arch}-v2/artifacts/model", tags=tags)
        await mlflow.set_alias(name, "champion", 2)
        t1 = time.perf_counter()

        async def settled():
            s = await cr_status()
            return s.get("phase") in ("Promoted", "RolledBack", "PromotionFailed") and s

        final = await wait_for(settled, timeout_s=timeout_s, poll_s=0.2)
        stop.set()
        await asyncio.gather(*bg)
        out["canary_predictor_gpus"] = {p.predictor: p.extra.get("gpus") for p in ctl.pods.values()}
        out.update(canary_phase=final.get("phase"), canary_seconds=round(time.perf_counter() - t1, 2),
                   current_version=final.get("currentModelVersion"),
                   rolled_back_version=final.get("rolledBackVersion"), error=final.get("error"),
                   last_gate=final.get("canaryLastGate"))
    sd = await kube.get(SELDON_GROUP, SELDON_VERSION, namespace, SELDON_PLURAL, name)
    out.update(served=served["n"], http_errors=served["errors"], by_predictor=served["by_predictor"],
               final_predictors={p["name"]: p["traffic"] for p in sd["spec"]["predictors"]},
               placement={k.split("/")[-1]: v for k, v in sd["spec"]["predictors"][0].get("annotations", {}).items()},
               events=[e["reason"] for e in kube.events], total_s=round(time.perf_counter() - t_start, 2))
    await op.stop()
    await ctl.stop()
    await scraper.stop()
    await prom_runner.cleanup()
    await reg_runner.cleanup()
    await mlflow.close()
    await prom.close()
    return out


if __name__ == "__main__":
    import argparse
    import json

    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="tiny-llama")
    ap.add_argument("--regress", choices=sorted(k for k in FAULTS if k), default=None)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--concurrency", type=int, default=8)
    ap.add_argument("--gpu-slots", type=int, default=None, help="predictors per GPU (default: 2 on a 1-GPU node)")
    ap.add_argument("--timeout", type=float, default=600.0)
    a = ap.parse_args()
    print(json.dumps(asyncio.run(run_llm_canary(a.arch, a.regress, a.device, concurrency=a.concurrency,
                                                gpu_slots=a.gpu_slots, timeout_s=a.timeout)), indent=2))
