"""Config 5's expert-parallel serving path on CPU: an MlflowModel CR asking for
``expertParallel: 2`` (``tensorParallel`` unset) becomes a predictor whose container command
is ``--ep 2`` on two GPUs of the node pool; the server launches two rank processes, each a
data-parallel engine over its shard of the experts (gloo all-to-all here, RCCL on GPUs), rank
0 serves HTTP and spreads requests over both engines (runtime/ep_serving.py).  Its /generate
tokens -- for sequential and concurrent requests -- equal an EP=1 predictor's on the same
Mixtral checkpoint (reference per-version predictor contract: mlflow_operator.py:194-238)."""
import asyncio

import pytest

transformers = pytest.importorskip("transformers")


def test_operator_deploys_ep2_predictor_matching_ep1(tmp_path):
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
    from test_loader_cpu import _tiny_mixtral

    ck = tmp_path / "1" / "run" / "artifacts" / "model"
    ck.mkdir(parents=True)
    _tiny_mixtral(ck)
    prompts = [[5, 9, 11, 40, 2, 7, 300, 12], list(range(20, 61)), [100, 3, 17], [9] * 20]

    async def go():
        kube, reg = FakeKube(), SqliteRegistry()
        reg.create_model_version("moe", f"file://{ck.parent}", tags={"mlop.runtime": seldon.RUNTIME_LLM})
        reg.set_alias("moe", "champion", 1)
        op, _ = make_operator(kube, LocalMlflowClient(reg), LocalProm(MetricStore()), RealClock(), OperatorSettings())
        pool = GpuPool(4)
        launcher = ProcessLauncher(ready_timeout_s=240, gpus=pool, extra_env={
            "MLOP_DEVICE": "cpu", "MLOP_DTYPE": "float32", "MLOP_ENGINE_USE_GRAPHS": "false",
            "MLOP_ENGINE_NUM_KV_BLOCKS": "64", "MLOP_ENGINE_MAX_MODEL_LEN": "256", "OMP_NUM_THREADS": "1"})
        ctl = FakeSeldonController(kube, launcher, RealClock()).start()
        await op.start()
        try:
            await kube.create(GROUP, VERSION, "ns", PLURAL, mlflow_model_cr("ep1", "ns", "moe", "champion"))
            await kube.create(GROUP, VERSION, "ns", PLURAL,
                              mlflow_model_cr("ep2", "ns", "moe", "champion", expertParallel=2))

            async def ready():
                objs = [await kube.get(GROUP, VERSION, "ns", PLURAL, n) for n in ("ep1", "ep2")]
                return all((o.get("status") or {}).get("ready") == "True" for o in objs)

            await wait_for(ready, 240)
            sd2 = await kube.get(SELDON_GROUP, SELDON_VERSION, "ns", SELDON_PLURAL, "ep2")
            pred = sd2["spec"]["predictors"][0]
            c = pred["componentSpecs"][0]["spec"]["containers"][0]
            assert c["args"][c["args"].index("--ep") + 1] == "2" and "--tp" not in c["args"]
            assert seldon.gpus_of(pred) == 2
            pods = {k[1]: p for k, p in ctl.pods.items()}
            assert len(pods["ep2"].extra["gpus"]) == 2
            out = {}
            async with aiohttp.ClientSession() as s:
                async def gen(name, ids):
                    async with s.post(pods[name].endpoint + "/v2/models/moe/generate",
                                      json={"input_ids": ids, "parameters": {"max_tokens": 6,
                                                                            "ignore_eos": True}}) as r:
                        assert r.status == 200, await r.text()
                        return (await r.json())["output_ids"]

                for name in ("ep1", "ep2"):
                    out[name] = [await gen(name, ids) for ids in prompts]
                # concurrent: the EP front spreads them over both ranks' engines
                out["ep2_conc"] = list(await asyncio.gather(*(gen("ep2", ids) for ids in prompts)))
                # bad requests fail alone (400, validated on rank 0 before any rank sees them) and
                # the group keeps serving: empty, longer than max_model_len, out-of-vocab, bad params
                bad = [({"input_ids": [], "parameters": {"max_tokens": 2}}),
                       ({"input_ids": [5] * 300, "parameters": {"max_tokens": 2}}),
                       ({"input_ids": [10 ** 9], "parameters": {"max_tokens": 2}}),
                       ({"input_ids": [5, 6], "parameters": {"max_tokens": 2, "top_p": 0}})]
                codes = []
                for body in bad:
                    async with s.post(pods["ep2"].endpoint + "/v2/models/moe/generate", json=body) as r:
                        codes.append(r.status)
                out["bad_codes"] = codes
                out["after_bad"] = [await gen("ep2", ids) for ids in prompts[:2]]
                async with s.get(pods["ep2"].endpoint + "/metrics") as r:
                    txt = await r.text()
            return out, txt
        finally:
            await ctl.stop()
            await op.stop()

    out, txt = asyncio.run(asyncio.wait_for(go(), 300))
    assert out["ep2"] == out["ep1"]
    assert out["ep2_conc"] == out["ep1"]
    assert out["bad_codes"] == [400, 400, 400, 400], out["bad_codes"]
    assert out["after_bad"] == out["ep1"][:2]
    assert all(len(o) == 6 for o in out["ep1"])
    assert "mlop_engine_steps_total{" in txt
