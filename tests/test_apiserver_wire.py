"""The operator's real-cluster code path over the wire (no cluster, no kind here):
``RestKube`` against the kube-apiserver front-end of ``FakeKube``
(``controller/apiserver.py``), and ``python -m mlopamd.controller run`` as a
separate process wired by KUBECONFIG / MLFLOW_TRACKING_URI / MLOP_PROMETHEUS_URL
to HTTP fakes of the apiserver, the MLflow registry and Prometheus.

Reference behavior pinned here: CR create -> status.currentModelVersion + a
SeldonDeployment owned by the CR with predictor ``v{ver}`` at 100 % traffic
(`mlflow_operator.py:104-118,159-238`); a new alias version -> two predictors at
90/10 (`:184-187`); CR delete -> SD garbage-collected (`:162-169`)."""
import asyncio
import os
import socket
import subprocess
import sys
import time

import pytest

from mlopamd.controller.apiserver import serve_apiserver, write_kubeconfig
from mlopamd.controller.crd import GROUP, PLURAL, SELDON_GROUP, SELDON_PLURAL, SELDON_VERSION, VERSION
from mlopamd.controller.kube import ApiError, FakeKube, RestKube
from mlopamd.controller.local import mlflow_model_cr
from mlopamd.controller.mlflow import SqliteRegistry, serve_registry
from mlopamd.controller.prometheus import MetricStore, serve_prometheus

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(coro):
    return asyncio.run(coro)


def test_restkube_crud_semantics_over_http():
    async def go():
        fk = FakeKube()
        runner, url = await serve_apiserver(fk, token="tok")
        k = RestKube(url, token="tok")
        try:
            cr = mlflow_model_cr("m1", "ns", "iris", "champion")
            cr["metadata"]["labels"] = {"team": "a"}
            made = await k.create(GROUP, VERSION, "ns", PLURAL, cr)
            assert made["metadata"]["uid"] and made["metadata"]["generation"] == 1
            with pytest.raises(ApiError) as e:
                await k.create(GROUP, VERSION, "ns", PLURAL, cr)
            assert e.value.status == 409 and e.value.reason == "AlreadyExists"
            got = await k.get(GROUP, VERSION, "ns", PLURAL, "m1")
            assert got["spec"]["modelAlias"] == "champion"
            assert [o["metadata"]["name"] for o in await k.list(GROUP, VERSION, "ns", PLURAL, {"team": "a"})] == ["m1"]
            assert await k.list(GROUP, VERSION, "ns", PLURAL, {"team": "b"}) == []
            # status subresource: status-only writes keep spec + generation
            st = await k.patch_status(GROUP, VERSION, "ns", PLURAL, "m1", {"status": {"currentModelVersion": "3"}})
            assert st["status"]["currentModelVersion"] == "3" and st["metadata"]["generation"] == 1
            # spec merge-patch bumps generation, status untouched by main-resource writes
            sp = await k.patch(GROUP, VERSION, "ns", PLURAL, "m1", {"spec": {"modelAlias": "canary"}})
            assert sp["metadata"]["generation"] == 2 and sp["status"]["currentModelVersion"] == "3"
            # optimistic concurrency: replace with a stale resourceVersion is a 409 Conflict
            stale = dict(got)
            with pytest.raises(ApiError) as e:
                await k.replace(GROUP, VERSION, "ns", PLURAL, "m1", stale)
            assert e.value.status == 409 and e.value.reason == "Conflict"
            # ownerReferences GC: deleting the CR deletes the SD it owns
            sd = {"apiVersion": f"{SELDON_GROUP}/{SELDON_VERSION}", "kind": "SeldonDeployment",
                  "metadata": {"name": "m1", "ownerReferences": [{"apiVersion": f"{GROUP}/{VERSION}",
                                                                  "kind": "MlflowModel", "name": "m1",
                                                                  "uid": made["metadata"]["uid"],
                                                                  "controller": True}]},
                  "spec": {"predictors": []}}
            await k.create(SELDON_GROUP, SELDON_VERSION, "ns", SELDON_PLURAL, sd)
            await k.create_event("ns", {"reason": "Test", "type": "Normal", "message": "x",
                                        "involvedObject": {"name": "m1", "kind": "MlflowModel"}})
            assert fk.events_for("m1", "Test")
            await k.delete(GROUP, VERSION, "ns", PLURAL, "m1")
            for g, v, p in ((GROUP, VERSION, PLURAL), (SELDON_GROUP, SELDON_VERSION, SELDON_PLURAL)):
                with pytest.raises(ApiError) as e:
                    await k.get(g, v, "ns", p, "m1")
                assert e.value.status == 404 and e.value.reason == "NotFound"
            # bearer token enforced
            bad = RestKube(url, token="nope")
            with pytest.raises(ApiError) as e:
                await bad.get(GROUP, VERSION, "ns", PLURAL, "m1")
            assert e.value.status == 401
            await bad.close()
        finally:
            await k.close()
            await runner.cleanup()
    run(go())


def test_restkube_watch_stream():
    async def go():
        fk = FakeKube()
        runner, url = await serve_apiserver(fk)
        k = RestKube(url)
        await k.create(GROUP, VERSION, "ns", PLURAL, mlflow_model_cr("pre", "ns", "iris", "champion"))
        seen = []

        async def consume():
            async for etype, obj in k.watch(GROUP, VERSION, PLURAL, "ns"):
                seen.append((etype, obj["metadata"]["name"]))
                if etype == "DELETED":
                    return

        task = asyncio.get_running_loop().create_task(consume())
        try:
            t0 = time.monotonic()
            while ("ADDED", "pre") not in seen and time.monotonic() - t0 < 10:
                await asyncio.sleep(0.02)
            await asyncio.sleep(0.1)  # the watch request is open
            await k.create(GROUP, VERSION, "ns", PLURAL, mlflow_model_cr("w", "ns", "iris", "champion"))
            await k.patch(GROUP, VERSION, "ns", PLURAL, "w", {"spec": {"monitoringInterval": 5}})
            await k.delete(GROUP, VERSION, "ns", PLURAL, "w")
            await asyncio.wait_for(task, 10)
        finally:
            task.cancel()
            await k.close()
            await runner.cleanup()
        assert seen[0] == ("ADDED", "pre")
        kinds = [t for t, n in seen if n == "w"]
        assert "ADDED" in kinds[:2] and "MODIFIED" in kinds and kinds[-1] == "DELETED"
    run(go())


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_operator_cli_over_the_wire(tmp_path):
    """`python -m mlopamd.controller run` (RestKube + MlflowRestClient + PromClient) as its
    own process against HTTP fakes: the deployment path a real cluster would see."""
    async def go():
        fk = FakeKube()
        kube_runner, kube_url = await serve_apiserver(fk, token="sa-token")
        reg = SqliteRegistry()
        reg.create_model_version("iris", "mlflow-artifacts:/1/abc/artifacts/model")
        reg.create_model_version("iris", "mlflow-artifacts:/1/def/artifacts/model")
        reg.set_alias("iris", "champion", 1)
        ml_runner, ml_url = await serve_registry(reg)
        prom_runner, prom_url = await serve_prometheus(MetricStore())
        kc = write_kubeconfig(tmp_path / "kubeconfig", kube_url, "sa-token")
        port = _free_port()
        env = dict(os.environ, KUBECONFIG=kc, MLFLOW_TRACKING_URI=ml_url, MLOP_PROMETHEUS_URL=prom_url,
                   PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
        log = open(tmp_path / "operator.log", "w")
        proc = subprocess.Popen([sys.executable, "-m", "mlopamd.controller", "run", "--namespace", "wire",
                                 "--port", str(port)], cwd=ROOT, env=env, stdout=log, stderr=subprocess.STDOUT)
        k = RestKube(kube_url, token="sa-token")

        async def until(pred, timeout=60.0):
            t0 = time.monotonic()
            while time.monotonic() - t0 < timeout:
                assert proc.poll() is None, (tmp_path / "operator.log").read_text()[-3000:]
                try:
                    v = await pred()
                except ApiError:
                    v = None
                if v:
                    return v
                await asyncio.sleep(0.1)
            raise AssertionError("timed out; operator log:\n" + (tmp_path / "operator.log").read_text()[-3000:])

        try:
            await k.create(GROUP, VERSION, "wire", PLURAL, mlflow_model_cr("iris-model", "wire", "iris", "champion"))

            async def sd_one():
                sd = await k.get(SELDON_GROUP, SELDON_VERSION, "wire", SELDON_PLURAL, "iris-model")
                return sd if len(sd["spec"]["predictors"]) == 1 else None
            sd = await until(sd_one)
            pred = sd["spec"]["predictors"][0]
            assert pred["name"] == "v1" and pred["traffic"] == 100
            assert pred["graph"]["modelUri"] == "s3://mlflow/1/abc/artifacts/model"
            assert sd["spec"]["protocol"] == "kfserving"
            assert sd["metadata"]["ownerReferences"][0]["kind"] == "MlflowModel"
            cr = await k.get(GROUP, VERSION, "wire", PLURAL, "iris-model")
            assert cr["status"]["currentModelVersion"] == "1"
            assert fk.events_for("iris-model", "NewModelVersionDetected")
            # operator pod endpoints
            import aiohttp
            async with aiohttp.ClientSession() as s:
                async with s.get(f"http://127.0.0.1:{port}/healthz") as r:
                    assert r.status == 200
            # new alias version: canary split 90/10 (old/new)
            reg.set_alias("iris", "champion", 2)
            await k.patch(GROUP, VERSION, "wire", PLURAL, "iris-model", {"spec": {"monitoringInterval": 1}})

            async def sd_two():
                sd = await k.get(SELDON_GROUP, SELDON_VERSION, "wire", SELDON_PLURAL, "iris-model")
                return sd if len(sd["spec"]["predictors"]) == 2 else None
            sd = await until(sd_two)
            traffic = {p["name"]: p["traffic"] for p in sd["spec"]["predictors"]}
            assert traffic == {"v1": 90, "v2": 10}
            cr = await k.get(GROUP, VERSION, "wire", PLURAL, "iris-model")
            assert cr["status"]["currentModelVersion"] == "2" and cr["status"]["previousModelVersion"] == "1"
            # CR delete -> the owned SD is garbage-collected
            await k.delete(GROUP, VERSION, "wire", PLURAL, "iris-model")
            with pytest.raises(ApiError):
                await k.get(SELDON_GROUP, SELDON_VERSION, "wire", SELDON_PLURAL, "iris-model")
        finally:
            proc.terminate()
            try:
                proc.wait(10)
            except subprocess.TimeoutExpired:
                proc.kill()
            log.close()
            await k.close()
            for r in (kube_runner, ml_runner, prom_runner):
                await r.cleanup()
    run(go())
