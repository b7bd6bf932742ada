"""The V2 runtime server (in-process, CPU): sklearn + LLM backends, executor
metrics, streaming, fault injection; and the config-1 end-to-end demo."""
import asyncio
import json

import numpy as np
import pytest
import torch

from mlopamd.runtime.backends import ByteTokenizer, LLMBackend, SklearnBackend, save_linear_model
from mlopamd.runtime.metrics import RuntimeMetrics
from mlopamd.runtime.server import make_app


def _client(app):
    from aiohttp.test_utils import TestClient, TestServer

    return TestClient(TestServer(app))


def test_sklearn_iris_v2_infer(tmp_path):
    from mlopamd.controller.demo import train_iris

    path, acc = train_iris(tmp_path / "m")
    b = SklearnBackend(f"file://{path}", name="iris")
    m = RuntimeMetrics("iris", "v1", "ns", "iris")
    from sklearn.datasets import load_iris

    X, y = load_iris(return_X_y=True)

    async def go():
        async with _client(make_app(b, m)) as c:
            r = await c.get("/v2/health/ready")
            assert r.status == 200
            r = await c.post("/v2/models/iris/infer", json={"inputs": [
                {"name": "input-0", "shape": [150, 4], "datatype": "FP64", "data": X.ravel().tolist()}]})
            body = await r.json()
            pred = np.asarray(body["outputs"][0]["data"])
            assert (pred == y).mean() == pytest.approx(acc)
            await c.post("/api/v1.0/feedback", json={"reward": 1})
            txt = await (await c.get("/metrics")).text()
            assert 'seldon_api_executor_client_requests_seconds_count{code="200",deployment_name="iris"' in txt
            assert 'service="feedback"' in txt
    asyncio.run(go())


def test_linear_model_binary_and_regression(tmp_path):
    p = save_linear_model(tmp_path / "b", [[1.0, -1.0]], [0.0], [0, 1])
    b = SklearnBackend(str(p))
    assert b.predict(np.array([[2.0, 1.0], [0.0, 3.0]])).tolist() == [1, 0]


@pytest.fixture(scope="module")
def llm_backend():
    from mlopamd.models import build_model
    from mlopamd.models.config import TINY_LLAMA
    from mlopamd.runtime.engine import Engine, EngineConfig

    torch.manual_seed(0)
    m = build_model(TINY_LLAMA, device="cpu", dtype=torch.float32)
    eng = Engine(m, EngineConfig(max_num_seqs=4, max_model_len=256, num_kv_blocks=64, use_graphs=False))
    b = LLMBackend(eng, RuntimeMetrics("llm", "v1", "ns", "tiny"), name="tiny").start()
    yield b
    b.stop()


def test_llm_generate_infer_stream(llm_backend):
    async def go():
        async with _client(make_app(llm_backend, llm_backend.metrics)) as c:
            r = await c.post("/v2/models/tiny/generate", json={"text_input": "hello", "parameters": {
                "max_tokens": 5, "ignore_eos": True}})
            body = await r.json()
            assert r.status == 200 and len(body["output_ids"]) == 5 and body["finish_reason"] == "length"
            ids = ByteTokenizer().encode("hello")
            r = await c.post("/v2/models/tiny/infer", json={"inputs": [
                {"name": "input_ids", "shape": [len(ids)], "datatype": "INT64", "data": ids}],
                "parameters": {"max_tokens": 5, "ignore_eos": True}})
            body2 = await r.json()
            assert body2["outputs"][0]["data"] == body["output_ids"]  # greedy: deterministic
            r = await c.post("/v2/models/tiny/generate_stream", json={"input_ids": ids, "parameters": {
                "max_tokens": 4, "ignore_eos": True}})
            events = [json.loads(line[6:]) for line in (await r.text()).split("\n\n") if line.startswith("data: ")]
            assert [e["token_id"] for e in events[:-1]] == body["output_ids"][:4] and events[-1]["done"]
            # concurrent requests batch together
            outs = await asyncio.gather(*(c.post("/v2/models/tiny/generate", json={
                "input_ids": [5 + i, 6, 7], "parameters": {"max_tokens": 3, "ignore_eos": True}}) for i in range(4)))
            assert all(o.status == 200 for o in outs)
            txt = await (await c.get("/metrics")).text()
            assert "mlop_time_to_first_token_seconds_count" in txt and "mlop_generated_tokens_total" in txt
            assert "mlop_engine_steps_total{" in txt and "mlop_engine_tokens_total{" in txt
            assert 'mlop_kv_cache_fill_failed{' in txt and "mlop_kv_cache_blocks{" in txt
            # engine step trace (Chrome trace events) and its summary
            tr = await (await c.get("/v2/debug/trace")).json()
            kinds = {e["name"] for e in tr["traceEvents"]}
            assert tr["traceEvents"] and kinds <= {"prefill", "mixed", "decode", "idle"} and "decode" in kinds
            assert all(e["dur"] >= 0 for e in tr["traceEvents"])
            summ = await (await c.get("/v2/debug/steps")).json()
            assert summ["steps"]["decode"]["steps"] > 0 and summ["stats"]["decode_tokens"] > 0
    asyncio.run(go())


def test_out_of_range_sampling_params_fail_alone(llm_backend):
    """A request whose integers cannot fit the sampler's int32 / int64 tensors (top_k 2**40,
    seed 2**64, huge stop ids / max_tokens) gets a 400 and leaves the engine loop serving."""
    async def go():
        async with _client(make_app(llm_backend, llm_backend.metrics)) as c:
            bad = [{"temperature": 1.0, "seed": 2**64}, {"max_tokens": 2**40}, {"stop_token_ids": [2**40]},
                   {"seed": -1}, {"top_k": -3}]
            for params in bad:
                r = await c.post("/v2/models/tiny/generate", json={"input_ids": [5, 6, 7], "parameters": params})
                assert r.status == 400, (params, r.status, await r.text())
            # top_k beyond int32 means "no bound": served as full-vocabulary sampling
            r = await c.post("/v2/models/tiny/generate", json={"input_ids": [5, 6, 7], "parameters": {
                "temperature": 1.0, "top_k": 2**40, "seed": 3, "max_tokens": 3, "ignore_eos": True}})
            assert r.status == 200 and len((await r.json())["output_ids"]) == 3
            r = await c.post("/v2/models/tiny/generate", json={"input_ids": [5, 6, 7], "parameters": {
                "max_tokens": 4, "ignore_eos": True}})
            assert r.status == 200 and len((await r.json())["output_ids"]) == 4
    asyncio.run(go())
    assert llm_backend.failure is None if hasattr(llm_backend, "failure") else True


def test_torch_profile_window(tmp_path):
    """MLOP_PROFILE_STEPS-style window: torch.profiler around engine steps a..b, Chrome trace written."""
    import torch

    from mlopamd.models import build_model
    from mlopamd.models.config import TINY_LLAMA
    from mlopamd.runtime.engine import Engine, EngineConfig
    from mlopamd.runtime.sampler import SamplingParams
    from mlopamd.runtime.tracing import TorchProfileWindow

    eng = Engine(build_model(TINY_LLAMA, device="cpu", dtype=torch.float32, seed=1),
                 EngineConfig(max_num_seqs=2, max_model_len=64, num_kv_blocks=16, use_graphs=False))
    eng.profile_window = TorchProfileWindow("1:3", str(tmp_path))
    eng.generate([[3, 4, 5]], SamplingParams(max_tokens=5, ignore_eos=True))
    files = list(tmp_path.glob("engine_steps_1_3_*.json"))
    assert files and json.loads(files[0].read_text())["traceEvents"]


def test_fault_injection_counts_errors(tmp_path):
    p = save_linear_model(tmp_path / "b", [[1.0, -1.0]], [0.0], [0, 1])
    b = SklearnBackend(str(p))
    m = RuntimeMetrics("d", "v2", "ns", "m")

    async def go():
        async with _client(make_app(b, m, inject_error_rate=1.0)) as c:
            r = await c.post("/v2/models/m/infer", json={"inputs": [{"name": "x", "shape": [1, 2],
                                                                      "datatype": "FP32", "data": [1, 2]}]})
            assert r.status == 500
            txt = await (await c.get("/metrics")).text()
            assert 'code="500"' in txt
    asyncio.run(go())


@pytest.mark.slow
def test_config1_demo_end_to_end():
    from mlopamd.controller.demo import run_demo

    out = asyncio.run(asyncio.wait_for(run_demo(60), 240))
    assert out["accuracy"] > 0.9 and out["canary_phase"] == "Promoted"
    assert out["final_predictors"] == {"v2": 100}
    assert out["events"][:2] == ["NewModelVersionDetected", "PredictorReady"]
    assert "PromotionComplete" in out["events"]


def _sd(name, model_uri, env):
    return {"apiVersion": "machinelearning.seldon.io/v1", "kind": "SeldonDeployment",
            "metadata": {"name": name},
            "spec": {"predictors": [{"name": "v1", "traffic": 100, "replicas": 1,
                                     "graph": {"name": "classifier-1", "implementation": "MLFLOW_SERVER",
                                               "modelUri": model_uri},
                                     "componentSpecs": [{"spec": {"containers": [
                                         {"name": "classifier-1",
                                          "env": [{"name": k, "value": v} for k, v in env.items()]}]}}]}]}}


def test_process_predictor_crash_is_detected_and_restarted(tmp_path):
    """A real runtime process (V2 server, CPU sklearn-style model) exits with 139 after 1 s:
    the fake Seldon controller's liveness probe reports it (SD status restarts / reason) and
    restarts it as a new process, like the kubelet would."""
    from mlopamd.controller import seldon
    from mlopamd.controller.kube import FakeKube
    from mlopamd.controller.local import FakeSeldonController, ProcessLauncher

    p = save_linear_model(tmp_path / "m", [[1.0, -1.0]], [0.0], [0, 1])

    async def go():
        kube = FakeKube()
        launcher = ProcessLauncher(ready_timeout_s=60)
        ctl = FakeSeldonController(kube, launcher)
        ctl.PROBE_PERIOD_S, ctl.BACKOFF_S = 0.3, 0.3
        ctl.start()
        await kube.create("machinelearning.seldon.io", "v1", "ns", "seldondeployments",
                          _sd("m", f"file://{p}", {"MLOP_RUNTIME": "mlop-sklearn",
                                                   "MLOP_INJECT_CRASH_AFTER_S": "1.0"}))
        key = ("ns", "m", "v1")
        pids = set()
        for _ in range(300):
            pod = ctl.pods.get(key)
            if pod is not None and pod.proc is not None and pod.ready:
                pids.add(pod.proc.pid)
            if pod is not None and pod.restarts >= 2 and len(pids) >= 2:
                break
            await asyncio.sleep(0.1)
        sd = await kube.get("machinelearning.seldon.io", "v1", "ns", "seldondeployments", "m")
        restarts, failed, reason = seldon.predictor_health(sd, "v1")
        await ctl.stop()
        assert len(pids) >= 2, pids
        assert restarts >= 1 and not failed and "139" in reason

    asyncio.run(asyncio.wait_for(go(), 90))


def test_process_predictor_start_failure_reports_failed(tmp_path):
    from mlopamd.controller import seldon
    from mlopamd.controller.kube import FakeKube
    from mlopamd.controller.local import FakeSeldonController, ProcessLauncher

    p = save_linear_model(tmp_path / "m", [[1.0, -1.0]], [0.0], [0, 1])

    async def go():
        kube = FakeKube()
        ctl = FakeSeldonController(kube, ProcessLauncher(ready_timeout_s=60)).start()
        await kube.create("machinelearning.seldon.io", "v1", "ns", "seldondeployments",
                          _sd("m", f"file://{p}", {"MLOP_RUNTIME": "mlop-sklearn",
                                                   "MLOP_INJECT_START_ERROR": "HIP out of memory"}))
        for _ in range(300):
            sd = await kube.get("machinelearning.seldon.io", "v1", "ns", "seldondeployments", "m")
            if (sd.get("status") or {}).get("state") == "Failed":
                break
            await asyncio.sleep(0.1)
        await ctl.stop()
        assert sd["status"]["state"] == "Failed"
        _, failed, reason = seldon.predictor_health(sd, "v1")
        assert failed and "exited" in reason and "HIP out of memory" in reason

    asyncio.run(asyncio.wait_for(go(), 90))


def test_gpu_telemetry_is_per_pod(monkeypatch):
    """Only the GPUs exported to the pod (HIP_VISIBLE_DEVICES) are reported."""
    from mlopamd.runtime import gpu_metrics

    node = [{"gpu": i, "busy_percent": 10.0 * i, "mem_used": 1e9 * i, "mem_total": 288e9, "power_w": 500.0,
             "source": "test"} for i in range(8)]
    monkeypatch.setattr(gpu_metrics, "_sample_all", lambda: node)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "2,5")
    assert [d["gpu"] for d in gpu_metrics.sample()] == [2, 5]
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("CUDA_VISIBLE_DEVICES", raising=False)
    assert len(gpu_metrics.sample()) == 8  # no device list: a node-level (dev box) view


def test_kernel_time_shares_exported():
    from mlopamd.runtime import gpu_metrics
    from mlopamd.runtime.metrics import RuntimeMetrics

    ev = [("void mlop::gemm_pp_kernel<0, false, false>(...)", 600.0), ("mlop::paged_attn_kernel<4>", 300.0),
          ("mlop::rmsnorm_wave_kernel<8, true>", 50.0), ("Cijk_Alik_Bljk_BBS", 0.0), ("memcpy", 50.0)]
    sh = gpu_metrics.shares_from_events(ev)
    assert abs(sum(sh.values()) - 1.0) < 1e-9 and sh["gemm"] == 0.6 and sh["attention"] == 0.3
    m = RuntimeMetrics(deployment="d", predictor="v1", namespace="n")
    m.update_kernel_shares(sh)
    txt = m.exposition().decode()
    assert 'mlop_kernel_time_fraction{' in txt and 'kernel="attention"' in txt


def test_hip_warmup_loads_torchs_own_runtime():
    """The predictor's start-up thread initialises HIP while torch imports (server._warm_hip).  It
    must load torch's OWN libamdhip64 (torch/lib): a second HIP runtime in the process (e.g. the
    system ROCm copy) would not be the one torch and _C.so launch on.  After the server module,
    torch and the extension are loaded, exactly one HIP runtime file is mapped."""
    import os
    import subprocess
    import sys

    code = ("import time, mlopamd.runtime.server as s; s.start_hip_warmup(); time.sleep(0.5); "
            "from mlopamd import ops; ops.load(); "
            "print(sorted({l.split()[-1] for l in open('/proc/self/maps') if 'amdhip' in l}))")
    env = {k: v for k, v in os.environ.items() if k not in ("MLOP_DEVICE", "MLOP_HIP_WARMUP")}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    import ast

    maps = ast.literal_eval(out.stdout.strip().splitlines()[-1])
    torch_lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    assert len(maps) == 1 and maps[0].startswith(torch_lib), maps


def test_engine_clock_and_tokens_come_from_one_snapshot():
    """the HTTP served rate pairs the engine clock with the token total taken
    at that same instant (one collector over one tuple), never a token count from another step."""
    from mlopamd.runtime.metrics import RuntimeMetrics
    from prometheus_client import generate_latest

    m = RuntimeMetrics(deployment="d", predictor="v1", namespace="ns")
    m.mark_step(7, 10.5)
    m.mark_step(0, 11.0)
    m.mark_step(5, 12.25)
    txt = generate_latest(m.registry).decode()
    vals = {ln.split("{")[0]: float(ln.rsplit(" ", 1)[1]) for ln in txt.splitlines()
            if ln.startswith("mlop_engine_") and "{" in ln}
    assert vals["mlop_engine_clock_seconds"] == 12.25 and vals["mlop_engine_tokens_at_clock"] == 12
    assert vals["mlop_engine_tokens_total"] == 12 and vals["mlop_engine_steps_total"] == 3


def test_stop_token_ids_are_bounded_for_every_backend():
    import pytest as _pytest
    from mlopamd.runtime.sampler import MAX_STOP_IDS, SamplingParams

    SamplingParams(stop_token_ids=list(range(MAX_STOP_IDS))).validate()
    with _pytest.raises(ValueError, match="stop_token_ids"):
        SamplingParams(stop_token_ids=list(range(MAX_STOP_IDS + 1))).validate()
