"""BASELINE config 1 end to end on CPU (no GPU, no cluster, no network):

sqlite MLflow registry (served over its REST API) holds an sklearn-iris model
(trained here, saved in the pickle-free JSON format) -> MlflowModel CR ->
operator -> SeldonDeployment -> fake Seldon controller starts a REAL runtime
server process (V2 protocol) -> weighted router sends predictions -> the fake
Prometheus scrapes the runtime's executor metrics -> a second model version
goes through the Prometheus-gated canary to 100 %.
"""
from __future__ import annotations

import asyncio
import tempfile
import time
from pathlib import Path

import numpy as np


def train_iris(out_dir: Path, seed: int = 0) -> tuple[Path, float]:
    from sklearn.datasets import load_iris
    from sklearn.linear_model import LogisticRegression

    from ..runtime.backends import save_linear_model

    X, y = load_iris(return_X_y=True)
    clf = LogisticRegression(max_iter=500, random_state=seed).fit(X, y)
    acc = float(clf.score(X, y))
    return save_linear_model(out_dir, clf.coef_, clf.intercept_, clf.classes_), acc


async def run_demo(n_requests: int = 200, canary: bool = True, namespace: str = "seldon") -> dict:
    from sklearn.datasets import load_iris

    from .app import OperatorMetrics, make_operator
    from .clock import RealClock
    from .crd import GROUP, PLURAL, SELDON_GROUP, SELDON_PLURAL, SELDON_VERSION, VERSION, OperatorSettings
    from .kube import FakeKube
    from .local import FakeSeldonController, ProcessLauncher, Router, mlflow_model_cr, wait_for
    from .mlflow import MlflowRestClient, SqliteRegistry, serve_registry
    from .prometheus import MetricStore, PromClient, Scraper, serve_prometheus

    t_start = time.perf_counter()
    tmp = Path(tempfile.mkdtemp(prefix="mlop-demo-"))
    p1, acc1 = train_iris(tmp / "artifacts" / "1")
    p2, acc2 = train_iris(tmp / "artifacts" / "2", seed=1)
    reg = SqliteRegistry(str(tmp / "mlflow.db"))
    reg_runner, reg_url = await serve_registry(reg)
    mlflow = MlflowRestClient(reg_url)
    await mlflow.create_registered_model("iris")
    await mlflow.create_model_version("iris", f"file://{p1}", tags={"mlop.runtime": "mlop-sklearn"})
    await mlflow.set_alias("iris", "champion", 1)

    clock = RealClock()
    store = MetricStore()
    scraper = Scraper(store, clock, interval_s=0.5)
    prom_runner, prom_url = await serve_prometheus(store)
    kube = FakeKube()
    metrics = OperatorMetrics()
    prom = PromClient(prom_url)
    op, rec = make_operator(kube, mlflow, prom, clock, OperatorSettings(), metrics=metrics)
    ctl = FakeSeldonController(kube, ProcessLauncher(scraper, extra_env={"MLOP_DEVICE": "cpu"}), clock).start()
    router = Router(ctl)
    scraper.start()
    await op.start()
    cr = mlflow_model_cr("iris", namespace, "iris", "champion", interval=2,
                         canary={"step": 30, "intervalSeconds": 2, "attemptDelaySeconds": 1,
                                 "maxAttempts": 20, "windowSeconds": 6, "errorRateFloor": 0.01,
                                 "latencyFloorSeconds": 0.005})
    t_cr = time.perf_counter()
    await kube.create(GROUP, VERSION, namespace, PLURAL, cr)

    async def cr_status():
        return (await kube.get(GROUP, VERSION, namespace, PLURAL, "iris")).get("status") or {}

    await wait_for(lambda: _ready(cr_status), timeout_s=120)
    cr_ready_s = time.perf_counter() - t_cr

    X, y = load_iris(return_X_y=True)
    import aiohttp

    served = {"n": 0, "correct": 0, "by_predictor": {}}
    stop = asyncio.Event()

    async def load(session, limit=None):
        i = 0
        while not stop.is_set() and (limit is None or i < limit):
            k = i % len(X)
            payload = {"inputs": [{"name": "input-0", "shape": [1, 4], "datatype": "FP64", "data": X[k].tolist()}]}
            code, body, pred = await router.post(namespace, "iris", "/v2/models/iris/infer", payload, session)
            if code == 200:
                served["n"] += 1
                served["correct"] += int(body["outputs"][0]["data"][0] == int(y[k]))
                served["by_predictor"][pred] = served["by_predictor"].get(pred, 0) + 1
            i += 1
            await asyncio.sleep(0.002)

    async with aiohttp.ClientSession() as session:
        await load(session, n_requests)
        out = {"config": "sklearn-iris / local sqlite MLflow / CPU", "cr_ready_s": round(cr_ready_s, 3),
               "accuracy": served["correct"] / max(1, served["n"]), "train_accuracy": acc1}
        if canary:
            bg = asyncio.get_running_loop().create_task(load(session))
            await mlflow.create_model_version("iris", f"file://{p2}", tags={"mlop.runtime": "mlop-sklearn"})
            await mlflow.set_alias("iris", "champion", 2)
            t0 = time.perf_counter()

            async def promoted():
                s = await cr_status()
                return s.get("phase") in ("Promoted", "RolledBack", "PromotionFailed") and s

            final = await wait_for(promoted, timeout_s=180, poll_s=0.1)
            stop.set()
            await bg
            out.update(canary_phase=final.get("phase"), canary_seconds=round(time.perf_counter() - t0, 2),
                       current_version=final.get("currentModelVersion"))
    sd = await kube.get(SELDON_GROUP, SELDON_VERSION, namespace, SELDON_PLURAL, "iris")
    out.update(served=served["n"], by_predictor=served["by_predictor"],
               final_predictors={p["name"]: p["traffic"] for p in sd["spec"]["predictors"]},
               events=[e["reason"] for e in kube.events], total_s=round(time.perf_counter() - t_start, 2))
    await op.stop()
    await ctl.stop()
    await scraper.stop()
    await prom_runner.cleanup()
    await reg_runner.cleanup()
    await mlflow.close()
    await prom.close()
    return out


async def _ready(cr_status):
    s = await cr_status()
    return s.get("ready") == "True"


if __name__ == "__main__":
    import json

    print(json.dumps(asyncio.run(run_demo()), indent=2))
