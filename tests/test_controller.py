"""Control-plane integration tests on the in-memory fakes with a VIRTUAL clock:
the reference's 540 s canary and 60 s polls run in milliseconds.

Covers SURVEY.md §3.2-3.6 / Appendix A: first deploy, canary promotion,
canary failure -> rollback (+ anti-flap), reference no-rollback mode, alias
removal, registry outage (no delete), operator restart mid-canary, 409 retry,
CR deletion GC, spec update restarting the daemon, readiness gating.
"""
import asyncio

import pytest

from mlopamd.controller import seldon
from mlopamd.controller.app import OperatorMetrics, make_operator
from mlopamd.controller.clock import VirtualClock
from mlopamd.controller.crd import (GROUP, PLURAL, SELDON_GROUP, SELDON_PLURAL, SELDON_VERSION, VERSION,
                                    OperatorSettings)
from mlopamd.controller.kube import FakeKube
from mlopamd.controller.local import FakeSeldonController, SimLauncher, mlflow_model_cr
from mlopamd.controller.mlflow import LocalMlflowClient, SqliteRegistry
from mlopamd.controller.prometheus import LocalProm, MetricStore, MetricsUnavailable

NS = "models"


class Env:
    def __init__(self, profiles=None, rollback=True, startup=None):
        self.kube = FakeKube()
        self.reg = SqliteRegistry()
        self.clock = VirtualClock()
        self.store = MetricStore()
        self.metrics = OperatorMetrics()
        self.profiles = profiles or {}
        self.launcher = SimLauncher(self.store, self.clock, self.profiles, rps=100, period=5)
        self.rollback = rollback

    async def start(self):
        self.op, self.rec = make_operator(self.kube, LocalMlflowClient(self.reg), LocalProm(self.store, self.clock),
                                          self.clock, OperatorSettings(), metrics=self.metrics)
        self.ctl = FakeSeldonController(self.kube, self.launcher, self.clock).start()
        await self.op.start()

    async def stop(self):
        await self.op.stop()
        await self.ctl.stop()

    def version(self, tags=None):
        mv = self.reg.create_model_version("m", f"mlflow-artifacts:/7/abc{len(self.profiles)}/artifacts/model",
                                           tags=tags or {})
        return mv.version

    async def create_cr(self, **spec):
        canary = spec.pop("canary", {})
        canary.setdefault("rollback", self.rollback)
        await self.kube.create(GROUP, VERSION, NS, PLURAL,
                               mlflow_model_cr("m", NS, "m", "champion", interval=60, canary=canary, **spec))

    async def status(self):
        return (await self.kube.get(GROUP, VERSION, NS, PLURAL, "m")).get("status") or {}

    async def sd(self):
        try:
            return await self.kube.get(SELDON_GROUP, SELDON_VERSION, NS, SELDON_PLURAL, "m")
        except Exception:  # noqa: BLE001
            return None

    async def run_until(self, cond, max_virtual_s=5000.0):
        start = self.clock.now()
        while self.clock.now() - start < max_virtual_s:
            if await cond():
                return True
            await self.clock.sleep(1.0)
        return False

    def reasons(self):
        return [e["reason"] for e in self.kube.events]


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 60))


def test_first_deploy_reference_contract():
    async def go():
        env = Env()
        v1 = env.version()
        env.reg.set_alias("m", "champion", v1)
        await env.start()
        await env.create_cr()
        assert await env.run_until(lambda: _ready(env))
        st = await env.status()
        assert st["currentModelVersion"] == "1" and st.get("previousModelVersion") is None and "error" not in st
        sd = await env.sd()
        assert sd["apiVersion"] == "machinelearning.seldon.io/v1" and sd["spec"]["protocol"] == "kfserving"
        owner = sd["metadata"]["ownerReferences"][0]
        assert owner["kind"] == "MlflowModel" and owner["controller"] and owner["blockOwnerDeletion"]
        (p,) = sd["spec"]["predictors"]
        assert p["name"] == "v1" and p["traffic"] == 100 and p["replicas"] == 1
        assert p["graph"] == {"name": "classifier-1", "implementation": "MLFLOW_SERVER",
                              "modelUri": "s3://mlflow/7/abc0/artifacts/model",
                              "envSecretRefName": "minio-secret", "children": []}
        assert env.reasons()[:2] == ["NewModelVersionDetected", "PredictorReady"]
        await env.stop()
    run(go())


async def _ready(env):
    return (await env.status()).get("ready") == "True"


async def _phase(env, *phases):
    return (await env.status()).get("phase") in phases


def test_canary_promotes_in_reference_steps():
    async def go():
        env = Env(profiles={"1": {"latency": 0.05}, "2": {"latency": 0.05}})
        env.reg.set_alias("m", "champion", env.version())
        await env.start()
        await env.create_cr()
        assert await env.run_until(lambda: _ready(env))
        env.reg.set_alias("m", "champion", env.version())
        seen = []

        async def track():
            sd = await env.sd()
            seen.append(seldon.traffic_of(sd))
            return await _phase(env, "Promoted")
        t0 = env.clock.now()
        assert await env.run_until(track, 3000)
        elapsed = env.clock.now() - t0
        # 10 -> 100 in +10 steps, >= 60 s apart (reference: >= 9 x 60 s)
        news = sorted({t.get("v2") for t in seen if t.get("v2")})
        assert news[0] == 10 and 100 in news and len(news) >= 9
        assert elapsed >= 8 * 60
        assert env.reasons().count("TrafficIncrease") == 8
        assert env.reasons()[-1] == "PromotionComplete"
        sd = await env.sd()
        assert [p["name"] for p in sd["spec"]["predictors"]] == ["v2"]
        st = await env.status()
        assert st["currentModelVersion"] == "2" and st["previousModelVersion"] == "1"
        await env.stop()
    run(go())


def test_canary_regression_rolls_back_and_does_not_flap():
    async def go():
        env = Env(profiles={"1": {"latency": 0.05}, "2": {"latency": 0.5}})
        env.reg.set_alias("m", "champion", env.version())
        await env.start()
        await env.create_cr()
        assert await env.run_until(lambda: _ready(env))
        env.reg.set_alias("m", "champion", env.version())
        assert await env.run_until(lambda: _phase(env, "RolledBack"), 3000)
        st = await env.status()
        assert st["currentModelVersion"] == "1" and st["rolledBackVersion"] == "2"
        assert "PromotionFailed" in env.reasons() and env.reasons()[-1] == "RollbackComplete"
        sd = await env.sd()
        assert seldon.traffic_of(sd) == {"v1": 100}
        # the alias still points at v2: it must NOT be redeployed (no flapping)
        n_new = env.reasons().count("NewModelVersionDetected")
        await env.clock.sleep(600)
        assert env.reasons().count("NewModelVersionDetected") == n_new
        assert seldon.traffic_of(await env.sd()) == {"v1": 100}
        # a NEW version is still picked up
        env.profiles["3"] = {"latency": 0.05}
        env.reg.set_alias("m", "champion", env.version())
        assert await env.run_until(lambda: _phase(env, "Promoted"), 3000)
        await env.stop()
    run(go())


@pytest.mark.parametrize("guards,expect", [(None, "RolledBack"), ({}, "Promoted")])
def test_gpu_guard_tpot_regression(guards, expect):
    """Same request latency, but the new LLM predictor's time per output token is
    40% worse: the default GPU-side guard (tpot_avg <= 1.10x) rolls it back;
    gpuGuards: {} restores the reference gate, which promotes."""
    async def go():
        base = {"latency": 0.05, "gpu_mem": 40e9, "gpu_power": 700.0}
        env = Env(profiles={"1": dict(base, tpot=0.010), "2": dict(base, tpot=0.014)})
        env.reg.set_alias("m", "champion", env.version())
        await env.start()
        canary = {} if guards is None else {"gpuGuards": guards}
        await env.create_cr(canary=canary)
        assert await env.run_until(lambda: _ready(env))
        env.reg.set_alias("m", "champion", env.version())
        assert await env.run_until(lambda: _phase(env, expect), 3000)
        if expect == "RolledBack":
            assert seldon.traffic_of(await env.sd()) == {"v1": 100}
            assert "tpot_avg" in (await env.status())["error"]
        await env.stop()
    run(go())


def test_gpu_guard_hbm_regression_rolls_back():
    async def go():
        env = Env(profiles={"1": {"latency": 0.05, "gpu_mem": 40e9}, "2": {"latency": 0.05, "gpu_mem": 80e9}})
        env.reg.set_alias("m", "champion", env.version())
        await env.start()
        await env.create_cr()
        assert await env.run_until(lambda: _ready(env))
        env.reg.set_alias("m", "champion", env.version())
        assert await env.run_until(lambda: _phase(env, "RolledBack"), 3000)
        await env.stop()
    run(go())


@pytest.mark.parametrize("new_attn,expect", [(0.30, "Promoted"), (0.60, "RolledBack")])
def test_kernel_share_guard(new_attn, expect):
    """The gate consumes the pods' kernel-time shares (mlop_kernel_time_fraction, the
    in-process profiler's rocprof-style classes): a version whose attention kernels take
    more than 1.5x the old share of device time is rolled back even with equal latency."""
    async def go():
        old = {"latency": 0.05, "kernel_shares": {"gemm": 0.65, "attention": 0.25, "other": 0.10}}
        new = {"latency": 0.05, "kernel_shares": {"gemm": 0.65 - (new_attn - 0.25), "attention": new_attn,
                                                  "other": 0.10}}
        env = Env(profiles={"1": old, "2": new})
        env.reg.set_alias("m", "champion", env.version())
        await env.start()
        await env.create_cr()
        assert await env.run_until(lambda: _ready(env))
        env.reg.set_alias("m", "champion", env.version())
        assert await env.run_until(lambda: _phase(env, "RolledBack", "Promoted"), 3000)
        st = await env.status()
        assert st["phase"] == expect
        if expect == "RolledBack":
            assert "attention_share" in st["error"]
        await env.stop()
    run(go())


def test_reference_mode_no_rollback_leaves_split():
    async def go():
        env = Env(profiles={"1": {"latency": 0.05}, "2": {"error_rate": 0.5, "latency": 0.05}}, rollback=False)
        env.reg.set_alias("m", "champion", env.version())
        await env.start()
        await env.create_cr()
        assert await env.run_until(lambda: _ready(env))
        env.reg.set_alias("m", "champion", env.version())
        assert await env.run_until(lambda: _phase(env, "PromotionFailed"), 3000)
        assert seldon.traffic_of(await env.sd()) == {"v1": 90, "v2": 10}
        # level-triggered ticks after the failure must keep that split (not hand v2 100 %)
        for _ in range(4):
            await env.clock.sleep(40.0)
            assert seldon.traffic_of(await env.sd()) == {"v1": 90, "v2": 10}
            assert await _phase(env, "PromotionFailed")
        assert "RollbackComplete" not in env.reasons()
        await env.stop()
    run(go())


def test_alias_removed_deletes_deployment():
    async def go():
        env = Env()
        env.reg.set_alias("m", "champion", env.version())
        await env.start()
        await env.create_cr()
        assert await env.run_until(lambda: _ready(env))
        env.reg.delete_alias("m", "champion")
        assert await env.run_until(lambda: _phase(env, "AliasNotFound"), 200)
        st = await env.status()
        assert st["error"] == "Alias 'champion' does not exist"
        assert st.get("currentModelVersion") is None and st.get("previousModelVersion") is None
        assert await env.sd() is None
        assert "AliasNotFound" in env.reasons()
        # alias back -> redeployed
        env.reg.set_alias("m", "champion", 1)
        assert await env.run_until(lambda: _ready(env), 200)
        await env.stop()
    run(go())


def test_registry_outage_keeps_serving():
    async def go():
        env = Env()
        env.reg.set_alias("m", "champion", env.version())
        await env.start()
        await env.create_cr()
        assert await env.run_until(lambda: _ready(env))
        env.reg.fail_mode = "unavailable"
        await env.clock.sleep(300)
        assert await env.sd() is not None  # the reference deleted it here
        assert "RegistryUnavailable" in env.reasons() and "AliasNotFound" not in env.reasons()
        env.reg.fail_mode = None
        await env.clock.sleep(120)
        assert "registryUnavailable" not in await env.status()
        await env.stop()
    run(go())


class _FlakyProm:
    """LocalProm that raises MetricsUnavailable while ``down`` (Prometheus outage)."""

    def __init__(self, inner):
        self.inner, self.down, self.calls = inner, False, 0

    async def query(self, q, at=None):
        self.calls += 1
        if self.down:
            raise MetricsUnavailable("connection refused")
        return await self.inner.query(q, at)

    async def close(self):
        pass


def test_metrics_outage_pauses_canary_without_rollback():
    """A Prometheus outage longer than the gate's 10 attempts x 10 s must not roll back a
    healthy canary (missing data from a live backend still counts as a failed attempt):
    the split holds, one MetricsUnavailable Warning, then promotion resumes."""
    async def go():
        env = Env(profiles={"1": {"latency": 0.05}, "2": {"latency": 0.05}})
        env.reg.set_alias("m", "champion", env.version())
        flaky = _FlakyProm(LocalProm(env.store, env.clock))
        env.op, env.rec = make_operator(env.kube, LocalMlflowClient(env.reg), flaky, env.clock,
                                        OperatorSettings(), metrics=env.metrics)
        env.ctl = FakeSeldonController(env.kube, env.launcher, env.clock).start()
        await env.op.start()
        await env.create_cr()
        assert await env.run_until(lambda: _ready(env))
        env.reg.set_alias("m", "champion", env.version())

        async def at_30():
            st = await env.status()
            return st.get("phase") == "Canary" and st.get("canaryTraffic", 0) >= 30
        assert await env.run_until(at_30, 2000)
        flaky.down = True
        split = seldon.traffic_of(await env.sd())
        await env.clock.sleep(600)  # 60 gate attempts' worth of outage
        st = await env.status()
        assert st["phase"] == "Canary" and st["metricsUnavailable"] == "True"
        assert seldon.traffic_of(await env.sd()) == split
        assert env.reasons().count("MetricsUnavailable") == 1
        assert "RollbackComplete" not in env.reasons() and "PromotionFailed" not in env.reasons()
        flaky.down = False
        assert await env.run_until(lambda: _phase(env, "Promoted"), 3000)
        assert "metricsUnavailable" not in await env.status()
        await env.stop()
    run(go())


def test_operator_restart_resumes_canary():
    async def go():
        env = Env(profiles={"1": {"latency": 0.05}, "2": {"latency": 0.05}})
        env.reg.set_alias("m", "champion", env.version())
        await env.start()
        await env.create_cr()
        assert await env.run_until(lambda: _ready(env))
        env.reg.set_alias("m", "champion", env.version())

        async def at_30():
            return (await env.status()).get("canaryTraffic", 0) >= 30
        assert await env.run_until(at_30, 2000)
        await env.op.stop()  # operator pod dies mid-canary
        await env.clock.sleep(30)
        env.op, env.rec = make_operator(env.kube, LocalMlflowClient(env.reg), LocalProm(env.store, env.clock),
                                        env.clock, OperatorSettings())
        await env.op.start()
        assert await env.run_until(lambda: _phase(env, "Promoted"), 3000)
        assert seldon.traffic_of(await env.sd()) == {"v2": 100}
        await env.stop()
    run(go())


def test_conflict_on_apply_is_retried():
    async def go():
        env = Env(profiles={"1": {}, "2": {}})
        env.reg.set_alias("m", "champion", env.version())
        await env.start()
        await env.create_cr()
        assert await env.run_until(lambda: _ready(env))
        env.kube.fail_next("replace", 409, times=2)
        env.reg.set_alias("m", "champion", env.version())
        assert await env.run_until(lambda: _phase(env, "Canary"), 300)
        assert await env.run_until(lambda: _has_two(env), 300)
        await env.stop()
    run(go())


async def _has_two(env):
    sd = await env.sd()
    return sd and len(sd["spec"]["predictors"]) == 2


def test_cr_delete_garbage_collects_sd():
    async def go():
        env = Env()
        env.reg.set_alias("m", "champion", env.version())
        await env.start()
        await env.create_cr()
        assert await env.run_until(lambda: _ready(env))
        await env.kube.delete(GROUP, VERSION, NS, PLURAL, "m")
        await env.clock.sleep(5)
        assert await env.sd() is None and not env.ctl.pods
        await env.stop()
    run(go())


def test_spec_update_switches_alias():
    async def go():
        env = Env()
        v1, v2 = env.version(), env.version()
        env.reg.set_alias("m", "champion", v1)
        env.reg.set_alias("m", "challenger", v2)
        await env.start()
        await env.create_cr(canary={"initialTraffic": 50, "step": 50})
        assert await env.run_until(lambda: _ready(env))
        await env.kube.patch(GROUP, VERSION, NS, PLURAL, "m", {"spec": {"modelAlias": "challenger"}})

        async def on_v2():
            return (await env.status()).get("currentModelVersion") == "2"
        assert await env.run_until(on_v2, 300)
        await env.stop()
    run(go())


def test_slow_predictor_gates_after_readiness():
    async def go():
        env = Env(profiles={"1": {}, "2": {"startup_s": 400}})
        env.reg.set_alias("m", "champion", env.version())
        await env.start()
        await env.create_cr()
        assert await env.run_until(lambda: _ready(env))
        env.reg.set_alias("m", "champion", env.version())
        await env.clock.sleep(350)  # the reference would have failed the canary by now (90 s budget)
        st = await env.status()
        assert st["phase"] == "Canary" and st.get("canaryAttempts", 0) == 0
        assert await env.run_until(lambda: _phase(env, "Promoted"), 3000)
        await env.stop()
    run(go())


def test_llm_runtime_predictor_gets_gpus_and_placement():
    async def go():
        env = Env()
        v = env.version(tags={"mlop.architecture": "llama3-70b"})
        env.reg.set_alias("m", "champion", v)
        await env.start()
        await env.create_cr(tensorParallel=8, maxModelLen=8192, maxNumSeqs=128)
        assert await env.run_until(lambda: _ready(env))
        (p,) = (await env.sd())["spec"]["predictors"]
        c = p["componentSpecs"][0]["spec"]["containers"][0]
        assert c["resources"]["limits"]["amd.com/gpu"] == "8"
        assert p["annotations"]["mlop.amd.com/runtime"] == "mlop-llm"
        assert p["annotations"]["mlop.amd.com/tensorParallel"] == "8"
        env_names = {e["name"]: e["value"] for e in c["env"]}
        assert env_names["PREDICTOR_ID"] == "v1" and env_names["SELDON_DEPLOYMENT_ID"] == "m"
        assert env_names["MLOP_ARCHITECTURE"] == "llama3-70b"
        await env.stop()
    run(go())


def _gpu_node(name, gpus, vram="288G"):
    return {"apiVersion": "v1", "kind": "Node",
            "metadata": {"name": name, "labels": {"amd.com/gpu.vram": vram}},
            "status": {"allocatable": {"amd.com/gpu": str(gpus), "cpu": "128"}}}


def test_placement_reads_node_capacity():
    """G2 node-aware: the planner reads Node allocatable amd.com/gpu and the labeller's VRAM,
    subtracts GPUs other SeldonDeployments hold, and marks a TP=8 70B predictor unplaceable on
    a node with 4 free GPUs (fits=false + reason), while an auto-planned one lands in them."""
    async def go():
        env = Env()
        await env.kube.create("", "v1", None, "nodes", _gpu_node("mi355x-0", 8))
        # another team's predictor already holds 4 of the 8 GPUs
        other = seldon.build_seldon_deployment("other", "team", {"metadata": {"name": "o", "uid": "u"}}, [
            seldon.build_predictor(1, "s3://x", None, 100, runtime=seldon.RUNTIME_LLM,
                                   placement={"tensorParallel": 4, "gpus": 4})])
        await env.kube.create(SELDON_GROUP, SELDON_VERSION, "team", SELDON_PLURAL, other)
        v = env.version(tags={"mlop.architecture": "llama3-70b"})
        env.reg.set_alias("m", "champion", v)
        await env.start()
        await env.create_cr(tensorParallel=8, maxModelLen=8192, maxNumSeqs=128)
        assert await env.run_until(lambda: _ready(env))
        (p,) = (await env.sd())["spec"]["predictors"]
        ann = p["annotations"]
        assert ann["mlop.amd.com/fits"] == "False" and ann["mlop.amd.com/node"] == "mi355x-0"
        # the reason quotes momentary free counts: CR status, never the SD spec
        assert "mlop.amd.com/reason" not in ann
        why = (await env.status())["placement"]["v1"]
        assert "needs 8 GPUs" in why and "4 of 8" in why
        await env.stop()

        env2 = Env()
        await env2.kube.create("", "v1", None, "nodes", _gpu_node("mi355x-0", 8))
        await env2.kube.create(SELDON_GROUP, SELDON_VERSION, "team", SELDON_PLURAL, other)
        v = env2.version(tags={"mlop.architecture": "llama3-70b"})
        env2.reg.set_alias("m", "champion", v)
        await env2.start()
        await env2.create_cr(maxModelLen=8192, maxNumSeqs=128)  # auto: smallest TP that fits HBM
        assert await env2.run_until(lambda: _ready(env2))
        (p,) = (await env2.sd())["spec"]["predictors"]
        ann = p["annotations"]
        assert ann["mlop.amd.com/fits"] == "True" and int(ann["mlop.amd.com/gpus"]) <= 4
        await env2.stop()
    run(go())


def _gpu_pod(name, node, gpus, phase="Running"):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "team"},
            "spec": {"nodeName": node, "containers": [{"name": "c", "resources": {"limits": {"amd.com/gpu": str(gpus)}}}]},
            "status": {"phase": phase}}


def test_placement_charges_gpus_per_node():
    """Two 8-GPU nodes: pods bound to node A hold 6 of its GPUs, node B has a finished pod only.
    Per-node accounting (pods' nodeName) picks node B with 8 free, so a TP=8 70B predictor fits;
    the old single-node model charged every request to one node."""
    async def go():
        env = Env()
        await env.kube.create("", "v1", None, "nodes", _gpu_node("node-a", 8))
        await env.kube.create("", "v1", None, "nodes", _gpu_node("node-b", 8))
        await env.kube.create("", "v1", "team", "pods", _gpu_pod("p1", "node-a", 4))
        await env.kube.create("", "v1", "team", "pods", _gpu_pod("p2", "node-a", 2))
        await env.kube.create("", "v1", "team", "pods", _gpu_pod("p3", "node-b", 8, phase="Succeeded"))
        v = env.version(tags={"mlop.architecture": "llama3-70b"})
        env.reg.set_alias("m", "champion", v)
        await env.start()
        cap = await env.rec.node_capacity()
        assert cap["node"] == "node-b" and cap["free_gpus"] == 8 and cap["accounting"] == "per-node", cap
        await env.create_cr(tensorParallel=8, maxModelLen=8192, maxNumSeqs=128)
        assert await env.run_until(lambda: _ready(env))
        (p,) = (await env.sd())["spec"]["predictors"]
        ann = p["annotations"]
        assert ann["mlop.amd.com/fits"] == "True" and ann["mlop.amd.com/node"] == "node-b", ann
        await env.stop()
    run(go())


def test_own_predictor_pods_do_not_move_the_placement():
    """after the first deploy, the model's OWN predictor pods (Seldon labels
    them ``seldon-deployment-id: <SD>``) are bound to the node.  A later reconcile must not
    charge them against the model: the SD is not replaced, the placement stays, and a canary's
    new version is planned with the old version's GPUs subtracted once."""
    async def go():
        env = Env()
        await env.kube.create("", "v1", None, "nodes", _gpu_node("mi355x-0", 8))
        v1 = env.version(tags={"mlop.architecture": "llama3-70b"})
        env.reg.set_alias("m", "champion", v1)
        await env.start()
        await env.create_cr(tensorParallel=4, maxModelLen=8192, maxNumSeqs=64)
        assert await env.run_until(lambda: _ready(env))
        sd = await env.sd()
        (p,) = sd["spec"]["predictors"]
        assert p["annotations"]["mlop.amd.com/fits"] == "True"
        rv = sd["metadata"]["resourceVersion"]
        # the predictor's pod is now scheduled on the node and holds its 4 GPUs; another team's
        # pod holds 2 more
        own = _gpu_pod("m-v1-0", "mi355x-0", 4)
        own["metadata"].update(namespace=NS, labels={"seldon-deployment-id": "m"})
        await env.kube.create("", "v1", NS, "pods", own)
        await env.kube.create("", "v1", "team", "pods", _gpu_pod("x", "mi355x-0", 2))
        cap = await env.rec.node_capacity(exclude=(NS, "m"))
        assert cap["free_gpus"] == 6, cap  # own pod not charged
        assert (await env.rec.node_capacity())["free_gpus"] == 2
        for _ in range(3):  # several level-triggered passes
            env.rec.kick(NS, "m")
            await env.clock.sleep(61.0)
        sd2 = await env.sd()
        assert sd2["metadata"]["resourceVersion"] == rv and sd2["spec"] == sd["spec"]
        await env.stop()
    run(go())


def test_canary_is_planned_with_the_running_versions_gpus_charged():
    """v1's placement is REUSED from its annotations (no node read for
    it), and node_capacity excludes the model's own pods, so the canary's v2 must be charged
    with v1's GPUs explicitly.  8-GPU node: v1 (TP=4) holds 4 through its own pod, another
    team 2 -> 2 left, so a TP=4 v2 does not fit (before the fix it was planned onto 6)."""
    async def go():
        env = Env()
        await env.kube.create("", "v1", None, "nodes", _gpu_node("mi355x-0", 8))
        v1 = env.version(tags={"mlop.architecture": "llama3-70b"})
        env.reg.set_alias("m", "champion", v1)
        await env.start()
        await env.create_cr(tensorParallel=4, maxModelLen=8192, maxNumSeqs=64)
        assert await env.run_until(lambda: _ready(env))
        own = _gpu_pod("m-v1-0", "mi355x-0", 4)
        own["metadata"].update(namespace=NS, labels={"seldon-deployment-id": "m"})
        await env.kube.create("", "v1", NS, "pods", own)
        await env.kube.create("", "v1", "team", "pods", _gpu_pod("x", "mi355x-0", 2))
        v2 = env.version(tags={"mlop.architecture": "llama3-70b"})
        env.reg.set_alias("m", "champion", v2)

        async def split():
            sd = await env.sd()
            return sd is not None and len(sd["spec"]["predictors"]) == 2

        assert await env.run_until(split)
        preds = {p["name"]: p for p in (await env.sd())["spec"]["predictors"]}
        assert preds["v1"]["annotations"]["mlop.amd.com/fits"] == "True"  # v1 keeps its placement
        assert preds["v2"]["annotations"]["mlop.amd.com/fits"] == "False", preds["v2"]["annotations"]
        why = (await env.status())["placement"]["v2"]
        assert "2 of 8" in why, why
        # the planner's notes are consumed by the pass that wrote them (no stale entries)
        assert (NS, "m") not in env.rec.placement_notes
        await env.stop()
    run(go())


def test_placement_uses_node_vram_label():
    from mlopamd.controller import placement

    small = placement.plan("llama3-70b", 8192, 16, hbm_gb=96.0)  # a 96 GB part: 70B needs TP >= 2
    assert small.tensorParallel >= 2 and small.fits
    p = placement.plan("llama3-70b", 8192, 16, free_gpus=0)
    assert not p.fits and "0 of 8" in p.reason


def test_invalid_spec_reports_error():
    async def go():
        env = Env()
        await env.start()
        await env.kube.create(GROUP, VERSION, NS, PLURAL,
                              {"apiVersion": "mlflow.nizepart.com/v1alpha1", "kind": "MlflowModel",
                               "metadata": {"name": "m"}, "spec": {"modelAlias": "x"}})
        await env.clock.sleep(5)
        st = await env.status()
        assert st["phase"] == "Invalid" and "modelName" in st["error"]
        await env.stop()
    run(go())


# ------------------------------------------------- failure detection / recovery --

def test_canary_oom_at_start_rolls_back_fast():
    """The new version's predictor dies while loading (GPU out of memory): the Seldon
    controller reports it Failed and the canary is rolled back at once, not after the
    30-minute readiness timeout; the old version keeps 100 % of the traffic."""
    async def go():
        env = Env(profiles={"1": {"latency": 0.05},
                            "2": {"fail_start": "HIP out of memory: tried to allocate 96.00 GiB"}})
        env.reg.set_alias("m", "champion", env.version())
        await env.start()
        await env.create_cr()
        assert await env.run_until(lambda: _ready(env))
        t0 = env.clock.now()
        env.reg.set_alias("m", "champion", env.version())
        assert await env.run_until(lambda: _phase(env, "RolledBack"), 600)
        assert env.clock.now() - t0 < 300  # well inside readyTimeoutSeconds (1800)
        st = await env.status()
        assert st["currentModelVersion"] == "1" and st["rolledBackVersion"] == "2"
        assert "out of memory" in st["error"] and any(
            "out of memory" in e.get("message", "") for e in env.kube.events)
        assert seldon.traffic_of(await env.sd()) == {"v1": 100}
        await env.stop()
    run(go())


def test_crashed_predictor_is_restarted_and_recovers():
    """The serving predictor segfaults once after 100 s: the controller's liveness probe
    marks it unavailable (CR ready=False, PredictorUnavailable, restart counted) and
    restarts it after the CrashLoopBackOff delay; the CR is ready again."""
    async def go():
        env = Env(profiles={"1": {"latency": 0.05, "crash_after_s": 100, "crashes": 1}})
        env.reg.set_alias("m", "champion", env.version())
        await env.start()
        await env.create_cr()
        assert await env.run_until(lambda: _ready(env))
        assert await env.run_until(lambda: _not_ready(env), 400)
        st = await env.status()
        assert st["predictorRestarts"] == 1
        assert "PredictorUnavailable" in env.reasons()
        assert await env.run_until(lambda: _ready(env), 400)
        assert env.reasons().count("PredictorReady") == 2
        restarts, failed, reason = seldon.predictor_health(await env.sd(), "v1")
        assert restarts == 1 and not failed and "139" in reason
        await env.stop()
    run(go())


def test_crash_looping_canary_rolls_back():
    """A new version that crashes 30 s after every start is restarted with backoff and
    rolled back as soon as it reaches maxRestarts (2 here), whatever its gate said."""
    async def go():
        env = Env(profiles={"1": {"latency": 0.05}, "2": {"latency": 0.05, "crash_after_s": 30}})
        env.reg.set_alias("m", "champion", env.version())
        await env.start()
        await env.create_cr(canary={"maxRestarts": 2})
        assert await env.run_until(lambda: _ready(env))
        env.reg.set_alias("m", "champion", env.version())
        assert await env.run_until(lambda: _phase(env, "RolledBack"), 2000)
        st = await env.status()
        assert st["currentModelVersion"] == "1" and "restarted 2 times" in st["error"]
        fail = [e for e in env.kube.events if e["reason"] == "PromotionFailed"]
        assert fail and "unhealthy" in fail[-1]["message"]
        assert seldon.traffic_of(await env.sd()) == {"v1": 100}
        await env.stop()
    run(go())


async def _not_ready(env):
    return (await env.status()).get("ready") == "False"
