"""Configs 4 and 5 AS THE OPERATOR SHIPS THEM, on one MI355X.

An ``MlflowModel`` CR with ``tensorParallel: 2`` (tiny Llama checkpoint) or ``expertParallel: 2``
(tiny Mixtral checkpoint) is reconciled into a SeldonDeployment whose predictor container is the
plain runtime command (``python -m mlopamd.runtime.server --tp 2`` / ``--ep 2``, ``amd.com/gpu:
2``).  The local Seldon stand-in (``ProcessLauncher(share_gpu=True)``: the one-GPU rehearsal of a
2-GPU pod) runs THAT command; the container process becomes the rank launcher WITHOUT touching
the GPU (no /dev/kfd descriptor), its two ranks share cuda:0 over gloo with the IPC kernels
(K15 all-reduce / EP exchange) forced, and rank 0 serves V2 HTTP.  A TP=1 / EP=1 predictor of
the same checkpoint runs beside it.  Oracle: each predictor's greedy tokens against the dense
fp32 recompute of the checkpoint (argmax or within a small logit gap: TP / EP change the bf16
summation order); for the first generated token of every prompt, the multi-rank predictor must
also agree with the single-rank one.  Reference contract: one predictor per model version
(/root/reference/mlflow_operator.py:194-222).
"""
import asyncio
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
transformers = pytest.importorskip("transformers")

PROMPTS = [[5, 9, 11, 40, 2, 7, 300, 12], list(range(20, 61)), [100, 3], list(range(300, 390))]
N_TOK = 8


def _fds(pid):
    out = []
    for f in os.listdir(f"/proc/{pid}/fd"):
        try:
            out.append(os.readlink(f"/proc/{pid}/fd/{f}"))
        except OSError:
            pass
    return out


def _deploy_pair(ck, multi_spec: dict):
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

    async def go():
        kube, reg = FakeKube(), SqliteRegistry()
        reg.create_model_version("tiny", f"file://{ck.parent}", tags={"mlop.runtime": seldon.RUNTIME_LLM})
        reg.set_alias("tiny", "champion", 1)
        op, _ = make_operator(kube, LocalMlflowClient(reg), LocalProm(MetricStore()), RealClock(), OperatorSettings())
        launcher = ProcessLauncher(ready_timeout_s=300, gpus=GpuPool(1, slots_per_gpu=2), share_gpu=True,
                                   extra_env={"MLOP_ENGINE_NUM_KV_BLOCKS": "64", "MLOP_ENGINE_MAX_MODEL_LEN": "256",
                                              "MLOP_ENGINE_MAX_NUM_SEQS": "8"})
        ctl = FakeSeldonController(kube, launcher, RealClock()).start()
        await op.start()
        try:
            await kube.create(GROUP, VERSION, "ns", PLURAL, mlflow_model_cr("one", "ns", "tiny", "champion"))
            await kube.create(GROUP, VERSION, "ns", PLURAL,
                              mlflow_model_cr("multi", "ns", "tiny", "champion", **multi_spec))

            async def ready():
                objs = [await kube.get(GROUP, VERSION, "ns", PLURAL, n) for n in ("one", "multi")]
                for n in ("one", "multi"):
                    try:
                        sd = await kube.get(SELDON_GROUP, SELDON_VERSION, "ns", SELDON_PLURAL, n)
                    except Exception:  # noqa: BLE001
                        continue
                    for p in sd["spec"]["predictors"]:
                        _, failed, reason = seldon.predictor_health(sd, p["name"])
                        assert not failed, f"{n}/{p['name']} failed to start: {reason}"
                return all((o.get("status") or {}).get("ready") == "True" for o in objs)

            await wait_for(ready, 300, poll_s=0.1)
            sd = await kube.get(SELDON_GROUP, SELDON_VERSION, "ns", SELDON_PLURAL, "multi")
            pred = sd["spec"]["predictors"][0]
            args = pred["componentSpecs"][0]["spec"]["containers"][0]["args"]
            pods = {k[1]: p for k, p in ctl.pods.items()}
            info = {"args": args, "gpus_requested": seldon.gpus_of(pred),
                    "launcher_fds": _fds(pods["multi"].proc.pid), "single_fds": _fds(pods["one"].proc.pid)}
            out = {}
            async with aiohttp.ClientSession() as s:
                async with s.get(pods["multi"].endpoint + "/v2/debug/startup") as r:
                    info["startup"] = await r.json()
                for name in ("one", "multi"):
                    out[name] = []
                    for ids in PROMPTS:
                        async with s.post(pods[name].endpoint + "/v2/models/tiny/generate",
                                          json={"input_ids": ids, "parameters": {"max_tokens": N_TOK,
                                                                                "ignore_eos": True}}) as r:
                            assert r.status == 200, await r.text()
                            out[name].append((await r.json())["output_ids"])
            return out, info
        finally:
            await ctl.stop()
            await op.stop()

    return asyncio.run(asyncio.wait_for(go(), 600))


def _check(ck, out, info, flag):
    from mlopamd.models.loader import load_pretrained
    from test_model_gpu import _check_greedy

    assert info["args"][info["args"].index(flag) + 1] == "2" and info["gpus_requested"] == 2
    la = info["startup"]["launcher"]
    assert la["ranks"] == 2 and la["share_gpu"] and not la["hip_warmup_started"] and not la["kfd_open"]
    assert la["torch_imported"] is False
    assert "/dev/kfd" not in info["launcher_fds"], info["launcher_fds"]  # the launcher, while serving
    assert "/dev/kfd" in info["single_fds"]  # (the check can see a GPU process: the TP=1 pod is one)
    dense = load_pretrained(ck, device=torch.device("cuda", 0), dtype=torch.float32)
    for name in ("one", "multi"):
        assert all(len(o) == N_TOK for o in out[name])
        _check_greedy(dense, PROMPTS, out[name])
    assert [o[0] for o in out["multi"]] == [o[0] for o in out["one"]]


def test_operator_deploys_tp2_pod_on_one_gpu(gpu, tmp_path):
    from test_loader_cpu import _tiny_llama

    ck = tmp_path / "1" / "run" / "artifacts" / "model"
    ck.mkdir(parents=True)
    _tiny_llama(ck)
    out, info = _deploy_pair(ck, {"tensorParallel": 2})
    _check(ck, out, info, "--tp")


def test_operator_deploys_ep2_pod_on_one_gpu(gpu, tmp_path):
    from test_loader_cpu import _tiny_mixtral

    ck = tmp_path / "1" / "run" / "artifacts" / "model"
    ck.mkdir(parents=True)
    _tiny_mixtral(ck)
    out, info = _deploy_pair(ck, {"expertParallel": 2})
    _check(ck, out, info, "--ep")
