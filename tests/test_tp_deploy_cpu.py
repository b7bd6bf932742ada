"""Config 4's control path on CPU: an MlflowModel CR asking for ``tensorParallel: 2`` becomes a
SeldonDeployment whose predictor container is the plain runtime command (``--tp 2``,
``amd.com/gpu: 2``); the local Seldon stand-in (ProcessLauncher) runs THAT command with two
GPUs from the node pool, the server launches its two rank processes itself (gloo here, RCCL on
GPUs), and the TP=2 predictor's /generate tokens equal a TP=1 predictor's on the same
checkpoint (reference per-version predictor contract: mlflow_operator.py:194-222)."""
import asyncio

import pytest

transformers = pytest.importorskip("transformers")


def test_operator_deploys_tp2_predictor_matching_tp1(tmp_path):
    import aiohttp

    from mlopamd.controller import seldon
    from mlopamd.controller.app import make_operator
    from mlopamd.controller.clock import RealClock
    from mlopamd.controller.crd import GROUP, PLURAL, SELDON_GROUP, SELDON_PLURAL, SELDON_VERSION, VERSION, \
        OperatorSettings
    from mlopamd.controller.kube import FakeKube
    from mlopamd.controller.local import FakeSeldonController, GpuPool, ProcessLauncher, mlflow_model_cr, wait_for
    from mlopamd.controller.mlflow import LocalMlflowClient, SqliteRegistry
    from mlopamd.controller.prometheus import LocalProm, MetricStore
    from test_loader_cpu import _tiny_llama

    ck = tmp_path / "1" / "run" / "artifacts" / "model"
    ck.mkdir(parents=True)
    _tiny_llama(ck)
    prompts = [[5, 9, 11, 40, 2, 7, 300, 12], list(range(20, 61))]

    async def go():
        kube, reg = FakeKube(), SqliteRegistry()
        reg.create_model_version("tiny", f"file://{ck.parent}", tags={"mlop.runtime": seldon.RUNTIME_LLM})
        reg.set_alias("tiny", "champion", 1)
        op, _ = make_operator(kube, LocalMlflowClient(reg), LocalProm(MetricStore()), RealClock(), OperatorSettings())
        pool = GpuPool(4)
        launcher = ProcessLauncher(ready_timeout_s=240, gpus=pool, extra_env={
            "MLOP_DEVICE": "cpu", "MLOP_DTYPE": "float32", "MLOP_ENGINE_USE_GRAPHS": "false",
            "MLOP_ENGINE_NUM_KV_BLOCKS": "64", "MLOP_ENGINE_MAX_MODEL_LEN": "256", "OMP_NUM_THREADS": "1"})
        ctl = FakeSeldonController(kube, launcher, RealClock()).start()
        await op.start()
        try:
            await kube.create(GROUP, VERSION, "ns", PLURAL, mlflow_model_cr("tp1", "ns", "tiny", "champion"))
            await kube.create(GROUP, VERSION, "ns", PLURAL,
                              mlflow_model_cr("tp2", "ns", "tiny", "champion", tensorParallel=2))

            async def ready():
                objs = [await kube.get(GROUP, VERSION, "ns", PLURAL, n) for n in ("tp1", "tp2")]
                return all((o.get("status") or {}).get("ready") == "True" for o in objs)

            await wait_for(ready, 240)
            sd2 = await kube.get(SELDON_GROUP, SELDON_VERSION, "ns", SELDON_PLURAL, "tp2")
            pred = sd2["spec"]["predictors"][0]
            c = pred["componentSpecs"][0]["spec"]["containers"][0]
            assert c["args"][c["args"].index("--tp") + 1] == "2"
            assert seldon.gpus_of(pred) == 2
            pods = {k[1]: p for k, p in ctl.pods.items()}
            assert len(pods["tp2"].extra["gpus"]) == 2 and len(pods["tp1"].extra["gpus"]) == 1
            assert not set(pods["tp2"].extra["gpus"]) & set(pods["tp1"].extra["gpus"])
            assert pool.free == 1
            out = {}
            async with aiohttp.ClientSession() as s:
                for name in ("tp1", "tp2"):
                    out[name] = []
                    for ids in prompts:
                        async with s.post(pods[name].endpoint + "/v2/models/tiny/generate",
                                          json={"input_ids": ids, "parameters": {"max_tokens": 6,
                                                                                "ignore_eos": True}}) as r:
                            assert r.status == 200, await r.text()
                            out[name].append((await r.json())["output_ids"])
            return out
        finally:
            await ctl.stop()
            await op.stop()
            assert pool.free == 4  # every pod's GPUs returned to the node

    out = asyncio.run(asyncio.wait_for(go(), 300))
    assert out["tp2"] == out["tp1"]
    assert all(len(o) == 6 for o in out["tp1"])


def test_gpu_pool_assignment():
    from mlopamd.controller.local import GpuPool

    p = GpuPool(2)
    a = p.acquire(2)
    assert a == [0, 1]
    with pytest.raises(RuntimeError, match="Insufficient amd.com/gpu"):
        p.acquire(1)
    p.release(a)
    shared = GpuPool(1, slots_per_gpu=2)
    assert shared.acquire(1) == [0] and shared.acquire(1) == [0]
    with pytest.raises(RuntimeError):
        shared.acquire(1)
    with pytest.raises(RuntimeError):  # a pod's ranks never share one device
        GpuPool(1, slots_per_gpu=4).acquire(2)
