"""Unit tests: URI rewrite, gate, PromQL engine, placement, SD builder, CRD
compatibility with the reference, fake apiserver semantics, REST clients."""
import asyncio
import math

import pytest
import yaml
from hypothesis import given, settings, strategies as st

from mlopamd.controller import crd, placement, prometheus, seldon
from mlopamd.controller.kube import ApiError, FakeKube, merge_patch
from mlopamd.controller.mlflow import (MlflowRestClient, NotFound, RegistryUnavailable, SqliteRegistry,
                                       serve_registry)
from mlopamd.controller.prometheus import (LocalProm, MetricStore, MetricsUnavailable, PromClient, evaluate,
                                           get_model_metrics,
                                           model_queries, serve_prometheus, should_promote)


# ------------------------------------------------------------- C2 / URIs --

@pytest.mark.parametrize("src,rel", [("mlflow-artifacts:/1/abc/artifacts/model", "1/abc/artifacts/model"),
                                     ("/1/abc/model", "1/abc/model"), ("1/abc", "1/abc"),
                                     ("mlflow-artifacts://x", "x")])
def test_extract_relative_path(src, rel):
    assert crd.extract_relative_path(src) == rel
    assert crd.artifact_uri(src) == f"s3://mlflow/{rel}"


# ------------------------------------------------------------- C11 gate --

def M(p95, er, avg):
    return {"latency_95th": p95, "error_rate": er, "latency_avg": avg}


TH = {"latency_95th": 0.05, "error_rate": 0.02, "latency_avg": 0.05}


def test_gate_reference_table():
    assert should_promote(M(1.0, 0.1, 0.5), M(1.0, 0.1, 0.5), TH).promote
    assert should_promote(M(1.05, 0.102, 0.525), M(1.0, 0.1, 0.5), TH).promote
    assert not should_promote(M(1.06, 0.1, 0.5), M(1.0, 0.1, 0.5), TH).promote
    assert not should_promote(M(1.0, 0.11, 0.5), M(1.0, 0.1, 0.5), TH).promote
    assert not should_promote(M(1.0, 0.1, 0.53), M(1.0, 0.1, 0.5), TH).promote
    # missing metrics never promote (mlflow_operator.py:430-434)
    assert not should_promote(M(None, 0.1, 0.5), M(1.0, 0.1, 0.5), TH).promote
    assert not should_promote(M(1.0, 0.1, 0.5), M(1.0, None, 0.5), TH).promote
    # zero-error baseline: reference demands exactly 0; the floor relaxes it
    assert not should_promote(M(1, 0.001, 1), M(1, 0.0, 1), TH).promote
    assert should_promote(M(1, 0.001, 1), M(1, 0.0, 1), TH, error_rate_floor=0.01).promote


finite = st.floats(min_value=1e-4, max_value=1e3, allow_nan=False)


@settings(max_examples=200, deadline=None)
@given(finite, finite, finite, st.floats(0, 1), st.floats(0, 1), st.floats(0, 0.5))
def test_gate_properties(a, b, c, e1, e2, t):
    old = M(a, e1, c)
    # identical metrics always promote; a regression beyond threshold never does
    assert should_promote(old, old, {"latency_95th": t, "error_rate": t, "latency_avg": t}).promote
    worse = M(a * (1 + t) * 1.01 + 1e-9, e1, c)
    assert not should_promote(worse, old, {"latency_95th": t, "error_rate": t, "latency_avg": t}).promote
    # monotone in thresholds
    new = M(b, e2, c)
    if should_promote(new, old, {"latency_95th": t, "error_rate": t, "latency_avg": t}).promote:
        assert should_promote(new, old, {"latency_95th": t + 0.1, "error_rate": t + 0.1, "latency_avg": t + 0.1}).promote


# ---------------------------------------------------------------- PromQL --

def hist_store(lbl, lat_counts, t0=1000.0, step=5.0, n=20):
    """Cumulative histogram samples: per step, lat_counts = {le: count increment}."""
    s = MetricStore()
    cum = {le: 0.0 for le in lat_counts}
    tot = sm = 0.0
    for i in range(n):
        for le, c in lat_counts.items():
            cum[le] += c
        tot = cum["+Inf"]
        sm += 0.1 * lat_counts["+Inf"]
        t = t0 + i * step
        for le, c in cum.items():
            s.add("seldon_api_executor_client_requests_seconds_bucket", dict(lbl, le=le), c, t)
        s.add("seldon_api_executor_client_requests_seconds_sum", lbl, sm, t)
        s.add("seldon_api_executor_client_requests_seconds_count", lbl, tot, t)
        s.add("seldon_api_executor_server_requests_seconds_count", dict(lbl, code="200", service="predictions"), tot * 0.9, t)
        s.add("seldon_api_executor_server_requests_seconds_count", dict(lbl, code="500", service="predictions"), tot * 0.1, t)
    return s, t0 + (n - 1) * step


class _At:
    def __init__(self, t):
        self.t = t

    def now(self):
        return self.t


def test_reference_queries_evaluate():
    lbl = {"deployment_name": "m", "predictor_name": "v2", "namespace": "ns"}
    # per step: 10 requests; 5 <= 0.05s, 9 <= 0.1s, 10 <= 0.5s
    s, t = hist_store(lbl, {"0.05": 5, "0.1": 9, "0.5": 10, "+Inf": 10})
    q = model_queries("m", "v2", "ns", 60)
    p95 = evaluate(q["latency_95th"], s, t)
    # rank 0.95*N falls in (0.1, 0.5]: 0.1 + 0.4 * (9.5-9)/(10-9) = 0.3
    assert abs(p95[0][1] - 0.3) < 1e-9
    total = evaluate(q["total_responses"], s, t)[0][1]
    err = evaluate(q["error_responses"], s, t)[0][1]
    assert abs(err / total - 0.1) < 1e-9
    # empty selection -> "or on() vector(0)" gives 0
    assert evaluate(model_queries("m", "v9", "ns")["total_responses"], s, t) == [({}, 0.0)]
    assert evaluate(model_queries("m", "v9", "ns")["latency_95th"], s, t) == []
    m = asyncio.run(get_model_metrics(LocalProm(s, _At(t)), "m", "v2", "ns", 60))
    assert abs(m["latency_95th"] - 0.3) < 1e-9 and abs(m["error_rate"] - 0.1) < 1e-9
    assert abs(m["latency_avg"] - 0.1) < 1e-9 and m["request_count"] > 0
    assert asyncio.run(get_model_metrics(LocalProm(s, _At(t)), "m", "v9", "ns", 60))["error_rate"] is None


def test_promql_misc():
    s = MetricStore()
    for i in range(10):
        s.add("x_total", {"a": "1", "b": "q"}, i * 2.0, 100.0 + i)
        s.add("x_total", {"a": "2", "b": "q"}, i * 1.0, 100.0 + i)
    assert evaluate("sum(rate(x_total[5s]))", s, 109)[0][1] == pytest.approx(3.0)
    assert {d["a"]: v for d, v in evaluate('sum by (a) (increase(x_total{b="q"}[9s]))', s, 109)} == {"1": 18.0, "2": 9.0}
    assert evaluate('x_total{a=~"1|2", a!="2"}', s, 109)[0][1] == 18.0
    assert evaluate("2 * 3 + 1", s, 109) == 7.0
    assert evaluate('max(x_total) / 2', s, 109)[0][1] == 9.0
    # counter reset handled
    s.add("y_total", {}, 10, 0)
    s.add("y_total", {}, 15, 1)
    s.add("y_total", {}, 3, 2)
    assert evaluate("increase(y_total[10s])", s, 2)[0][1] == 8.0


def test_fake_prometheus_http_roundtrip():
    async def go():
        lbl = {"deployment_name": "m", "predictor_name": "v1", "namespace": "ns"}
        s, t = hist_store(lbl, {"0.05": 5, "0.1": 9, "0.5": 10, "+Inf": 10})
        runner, url = await serve_prometheus(s)
        c = PromClient(url)
        res = await c.query(model_queries("m", "v1", "ns")["latency_95th"], at=t)
        assert abs(float(res[0]["value"][1]) - 0.3) < 1e-9
        with pytest.raises(MetricsUnavailable):  # a query error is not "no samples"
            await c.query("bogus((", at=t)
        await c.close()
        await runner.cleanup()
        c2 = PromClient(url, timeout_s=2.0)
        with pytest.raises(MetricsUnavailable):  # nothing listening any more
            await c2.query("up")
        await c2.close()
    asyncio.run(go())


def test_exposition_ingest():
    from mlopamd.runtime.metrics import RuntimeMetrics

    m = RuntimeMetrics("dep", "v3", "ns", "model")
    for _ in range(8):
        m.observe_request(0.02, 200)
    m.observe_request(0.2, 500)
    m.observe_request(0.01, 200, service="feedback")
    s = MetricStore()
    s.ingest_exposition(m.exposition().decode(), 100.0)
    for _ in range(4):
        m.observe_request(0.02, 200)
    s.ingest_exposition(m.exposition().decode(), 130.0)
    mm = asyncio.run(get_model_metrics(LocalProm(s, _At(130.0)), "dep", "v3", "ns", 60))
    assert mm["request_count"] == 4.0 and mm["error_rate"] == 0.0
    fb = evaluate(model_queries("dep", "v3", "ns")["feedback"], s, 130.0)
    assert fb[0][1] == 0.0


# ------------------------------------------------------------- placement --

def test_placement_8b_fits_one_gpu():
    p = placement.plan("llama3-8b", 4096, 256)
    assert p.tensorParallel == 1 and p.gpus == 1 and p.fits and p.weightGBPerGPU == pytest.approx(16.06, 0.01)


def test_placement_70b():
    p = placement.plan("llama3-70b", 8192, 16)
    assert p.fits and p.tensorParallel == 1  # 141 GB + 43 GB KV fits one 288 GB GPU
    # worst-case KV (fraction 1.0): 171 GB for 64 x 8192 does not fit beside 141 GB of weights
    assert placement.plan("llama3-70b", 8192, 64, kv_target_fraction=1.0).tensorParallel == 2
    assert placement.plan("llama3-70b", 8192, 128).tensorParallel == 2  # mean-context target, 171 GB
    big = placement.plan("llama3-70b", 8192, 512)
    assert big.tensorParallel >= 2 and big.fits
    p8 = placement.plan("llama3-70b", 8192, 128, requested_tp=8)
    assert p8.tensorParallel == 8 and p8.gpus == 8 and p8.weightGBPerGPU < 18 and p8.fits
    assert not placement.plan("llama3-70b", requested_tp=3).fits


def test_placement_bench_config_is_one_gpu():
    """The headline bench (2048 concurrent x 1024 max len) is one 288 GB GPU per replica."""
    p = placement.plan("llama3-8b", 1024, 2048)
    assert p.tensorParallel == 1 and p.fits and p.kvTokenCapacity >= 2048 * 512


def test_placement_mixtral_ep():
    p = placement.plan("mixtral-8x7b", 4096, 256, requested_tp=8)
    assert p.expertParallel == 8 and p.gpus == 8


# ------------------------------------------------------------------- SD --

BODY = {"apiVersion": "mlflow.nizepart.com/v1alpha1", "kind": "MlflowModel",
        "metadata": {"name": "iris", "namespace": "ns", "uid": "u-1"}}


def test_sd_reference_shape():
    preds = [seldon.build_predictor("3", "s3://mlflow/a", "minio", 90),
             seldon.build_predictor("4", "s3://mlflow/b", "minio", 10)]
    sd = seldon.build_seldon_deployment("iris", "ns", BODY, preds)
    assert sd == {
        "apiVersion": "machinelearning.seldon.io/v1", "kind": "SeldonDeployment",
        "metadata": {"name": "iris", "namespace": "ns", "labels": {"app.kubernetes.io/managed-by": "mlflow-operator"},
                     "ownerReferences": [{"apiVersion": "mlflow.nizepart.com/v1alpha1", "kind": "MlflowModel",
                                          "name": "iris", "uid": "u-1", "controller": True, "blockOwnerDeletion": True}]},
        "spec": {"name": "iris", "protocol": "kfserving", "predictors": [
            {"graph": {"name": "classifier-3", "implementation": "MLFLOW_SERVER", "modelUri": "s3://mlflow/a",
                       "envSecretRefName": "minio", "children": []}, "name": "v3", "replicas": 1, "traffic": 90},
            {"graph": {"name": "classifier-4", "implementation": "MLFLOW_SERVER", "modelUri": "s3://mlflow/b",
                       "envSecretRefName": "minio", "children": []}, "name": "v4", "replicas": 1, "traffic": 10}]}}
    assert seldon.traffic_of(sd) == {"v3": 90, "v4": 10}
    assert not seldon.predictor_ready(sd, "v3")
    sd["status"] = {"state": "Available", "deploymentStatus": {"iris-v3-0-classifier-3": {"replicas": 1, "availableReplicas": 1}}}
    assert seldon.predictor_ready(sd, "v3") and not seldon.predictor_ready(sd, "v4")


# ------------------------------------------------------------------ CRD --

def test_crd_compatible_with_reference_fields():
    ours = crd.load_manifest("crd.yaml")[0]
    assert ours["metadata"]["name"] == "mlflowmodels.mlflow.nizepart.com"
    s = ours["spec"]
    assert (s["group"], s["scope"], s["names"]["kind"], s["names"]["plural"], s["names"]["singular"],
            s["names"]["shortNames"]) == ("mlflow.nizepart.com", "Namespaced", "MlflowModel", "mlflowmodels",
                                          "mlflowmodel", ["mlflowm"])
    v = s["versions"][0]
    assert v["name"] == "v1alpha1" and v["served"] and v["storage"] and v["subresources"] == {"status": {}}
    props = v["schema"]["openAPIV3Schema"]["properties"]
    for f, t in {"modelName": "string", "modelAlias": "string", "monitoringInterval": "integer",
                 "minioSecret": "string"}.items():
        assert props["spec"]["properties"][f]["type"] == t
    for f in ("currentModelVersion", "previousModelVersion", "error"):
        assert props["status"]["properties"][f]["type"] == "string"
    spec = crd.ModelSpec.from_spec({"modelName": "a", "modelAlias": "b"})
    assert spec.monitoring_interval == 60 and spec.canary.step == 10 and spec.canary.initial_traffic == 10
    assert spec.canary.interval_s == 60 and spec.canary.max_attempts == 10 and spec.canary.attempt_delay_s == 10


def test_rbac_and_deployment_manifests():
    docs = crd.load_manifest("rbac.yaml")
    role = next(d for d in docs if d["kind"] == "ClusterRole")
    rules = {tuple(r["resources"]): set(r["verbs"]) for r in role["rules"]}
    assert {"get", "list", "watch", "create", "update", "patch"} <= rules[("mlflowmodels", "mlflowmodels/status")]
    assert "delete" in rules[("seldondeployments", "seldondeployments/status")]
    assert {"create", "patch"} <= rules[("events",)]
    dep = crd.load_manifest("operator-deployment.yaml")[0]
    tpl = dep["spec"]["template"]["spec"]
    assert tpl["serviceAccountName"] == "mlflow-operator" and dep["spec"]["replicas"] == 1
    assert tpl["containers"][0]["envFrom"] == [{"secretRef": {"name": "mlflow-creds"}}]
    assert crd.load_manifest("namespace.yaml")[0]["metadata"]["name"] == "mlflow-operator"


# ------------------------------------------------------------ FakeKube --

def test_fake_kube_semantics():
    async def go():
        k = FakeKube()
        o = await k.create("mlflow.nizepart.com", "v1alpha1", "ns", "mlflowmodels",
                           {"metadata": {"name": "a"}, "spec": {"modelName": "m", "modelAlias": "c", "x": 1},
                            "status": {"s": 1}})
        assert "x" not in o["spec"]  # undeclared field pruned like the apiserver does
        assert "status" not in o and o["metadata"]["generation"] == 1
        o2 = await k.patch_status("mlflow.nizepart.com", "v1alpha1", "ns", "mlflowmodels", "a",
                                  {"status": {"currentModelVersion": "1", "error": None}})
        assert o2["status"] == {"currentModelVersion": "1"} and o2["metadata"]["generation"] == 1
        o3 = await k.patch("mlflow.nizepart.com", "v1alpha1", "ns", "mlflowmodels", "a",
                           {"spec": {"monitoringInterval": 30}, "status": {"hack": 1}})
        assert o3["metadata"]["generation"] == 2 and "hack" not in o3["status"]
        with pytest.raises(ApiError) as e:  # schema violation: 422 Invalid, nothing stored
            await k.patch("mlflow.nizepart.com", "v1alpha1", "ns", "mlflowmodels", "a",
                          {"spec": {"tensorParallel": 9, "monitoringInterval": "soon"}})
        assert e.value.status == 422 and "tensorParallel" in e.value.message and "monitoringInterval" in e.value.message
        with pytest.raises(ApiError) as e:
            await k.patch_status("mlflow.nizepart.com", "v1alpha1", "ns", "mlflowmodels", "a",
                                 {"status": {"canaryTraffic": "ten"}})
        assert e.value.status == 422
        stale = dict(o, spec={"modelName": "m", "modelAlias": "d"})
        with pytest.raises(ApiError) as e:
            await k.replace("mlflow.nizepart.com", "v1alpha1", "ns", "mlflowmodels", "a", stale)
        assert e.value.status == 409
        await k.create("machinelearning.seldon.io", "v1", "ns", "seldondeployments",
                       {"metadata": {"name": "a", "ownerReferences": [{"uid": o["metadata"]["uid"]}]}, "spec": {}})
        await k.delete("mlflow.nizepart.com", "v1alpha1", "ns", "mlflowmodels", "a")
        with pytest.raises(ApiError):
            await k.get("machinelearning.seldon.io", "v1", "ns", "seldondeployments", "a")
    asyncio.run(go())
    assert merge_patch({"a": 1, "b": {"c": 2}}, {"b": {"c": None, "d": 3}, "a": None}) == {"b": {"d": 3}}


# --------------------------------------------------------------- MLflow --

def test_mlflow_rest_against_sqlite_registry(tmp_path):
    async def go():
        reg = SqliteRegistry(str(tmp_path / "m.db"))
        runner, url = await serve_registry(reg)
        c = MlflowRestClient(url)
        await c.create_registered_model("m")
        mv = await c.create_model_version("m", "mlflow-artifacts:/1/x/artifacts/model", tags={"mlop.architecture": "llama3-8b"})
        assert mv.version == "1" and mv.tags["mlop.architecture"] == "llama3-8b"
        await c.set_alias("m", "champion", 1)
        got = await c.get_model_version_by_alias("m", "champion")
        assert got.version == "1" and got.source.endswith("artifacts/model") and "champion" in got.aliases
        with pytest.raises(NotFound):
            await c.get_model_version_by_alias("m", "nope")
        with pytest.raises(NotFound):
            await c.get_model_version("m", 9)
        reg.fail_mode = "unavailable"
        with pytest.raises(RegistryUnavailable):
            await c.get_model_version_by_alias("m", "champion")
        await c.close()
        await runner.cleanup()
        dead = MlflowRestClient("http://127.0.0.1:9", timeout_s=1)
        with pytest.raises(RegistryUnavailable):
            await dead.get_model_version("m", 1)
        await dead.close()
    asyncio.run(go())


def test_over_time_functions_and_gpu_guard_queries():
    st = prometheus.MetricStore()
    lbl = {"deployment_name": "d", "predictor_name": "v1", "namespace": "n"}
    for i, v in enumerate((10.0, 30.0, 20.0)):
        st.add("mlop_gpu_memory_used_bytes", dict(lbl, gpu="0"), v, 100.0 + 10 * i)
        st.add("mlop_gpu_power_watts", dict(lbl, gpu="0"), 100.0 * (i + 1), 100.0 + 10 * i)
        st.add("mlop_time_per_output_token_seconds_sum", lbl, 0.02 * 100 * i, 100.0 + 10 * i)
        st.add("mlop_time_per_output_token_seconds_count", lbl, 100.0 * i, 100.0 + 10 * i)
    q = prometheus.gpu_guard_queries("d", "v1", "n", 60)
    ev = lambda s: prometheus.evaluate(s, st, 121.0)  # noqa: E731
    assert ev(q["gpu_memory_used"])[0][1] == 30.0
    assert ev(q["gpu_power"])[0][1] == pytest.approx(200.0)
    assert ev(q["tpot_avg"])[0][1] == pytest.approx(0.02)
    assert ev('last_over_time(mlop_gpu_memory_used_bytes{predictor_name="v1"}[60s])')[0][1] == 20.0
    other = prometheus.gpu_guard_queries("d", "v9", "n", 60)
    assert ev(other["tpot_avg"]) == [] and ev(other["gpu_memory_used"]) == []


def test_gate_gpu_guards_skip_missing_series():
    base = {"latency_95th": 0.1, "error_rate": 0.0, "latency_avg": 0.05}
    g = prometheus.should_promote(dict(base, tpot_avg=0.02), dict(base, tpot_avg=0.01), {}, 0.0,
                                  extra_max_ratio={"tpot_avg": 1.1})
    assert not g.promote and "tpot_avg" in g.reasons[0]
    g = prometheus.should_promote(dict(base, tpot_avg=None), dict(base, tpot_avg=0.01), {}, 0.0,
                                  extra_max_ratio={"tpot_avg": 1.1})
    assert g.promote


def test_example_crs_admit_and_place():
    """manifests/examples: one CR per BASELINE config; each passes the CRD's
    structural schema unchanged (nothing pruned) and its GPU placement fits."""
    import glob
    import os

    files = sorted(glob.glob(os.path.join(str(crd.MANIFESTS), "examples", "*.yaml")))
    assert len(files) == 5, files
    schema = crd.crd_schema()
    for f in files:
        with open(f) as fh:
            (cr,) = [d for d in yaml.safe_load_all(fh) if d]
        pruned, errs = crd.admit(cr, schema)
        assert errs == [] and pruned == cr, (f, errs)
        spec = crd.ModelSpec.from_spec(cr["spec"])
        assert spec.validate() == []
        if spec.architecture:
            p = placement.plan(spec.architecture, max_model_len=spec.max_model_len or 4096,
                               max_num_seqs=spec.max_num_seqs or 256, requested_tp=spec.tensor_parallel,
                               requested_ep=spec.expert_parallel)
            assert p.fits, (f, p)
    bad = {"apiVersion": "mlflow.nizepart.com/v1alpha1", "kind": "MlflowModel", "metadata": {"name": "x"},
           "spec": {"modelName": "m", "modelAlias": "a", "tensorParallel": 0, "canary": {"step": "10"}}}
    _, errs = crd.admit(bad, schema)
    assert any("tensorParallel" in e for e in errs) and any("canary.step" in e for e in errs)
