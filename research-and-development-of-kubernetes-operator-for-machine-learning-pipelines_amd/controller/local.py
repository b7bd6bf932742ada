"""Local "cluster" emulator (no kind / kubectl / network in this environment).

  FakeKube (apiserver)  <->  Operator (our reconciler)  ->  SeldonDeployment
                                                              |
  FakeSeldonController: watches SDs, starts one "pod" per predictor through a
  Launcher, reports per-predictor availability in the SD status (what the real
  Seldon controller does), and keeps the traffic split for the Router
  (weighted routing = the Istio VirtualService stand-in).

Launchers:
  * ``InProcessLauncher`` — builds the predictor backend in this process (the
    bench: the Llama-3-8B engine on this rank's GPU);
  * ``ProcessLauncher``  — starts ``python -m mlopamd.runtime.server`` with the
    container env from the SD, scraped by the fake Prometheus;
  * ``SimLauncher``      — simulated predictors that write executor metrics into a
    MetricStore with a per-version latency/error profile (virtual-clock canary tests).
"""
from __future__ import annotations

import asyncio
import itertools
import json
import logging
import os
import socket
import subprocess
import sys
import time
from dataclasses import dataclass, field

from . import seldon
from .clock import RealClock
from .crd import API_VERSION, GROUP, KIND, PLURAL, SELDON_GROUP, SELDON_PLURAL, SELDON_VERSION, VERSION
from .kube import ApiError, FakeKube

log = logging.getLogger("mlopamd.local")


@dataclass
class Pod:
    sd: str
    namespace: str
    predictor: str
    spec: dict
    endpoint: str | None = None
    backend: object = None
    ready: bool = False
    proc: subprocess.Popen | None = None
    task: asyncio.Task | None = None
    extra: dict = field(default_factory=dict)
    restarts: int = 0
    last_error: str = ""

    @property
    def key(self):
        return (self.namespace, self.sd, self.predictor)


def _env_of(pred: dict) -> dict:
    env = {}
    for cs in pred.get("componentSpecs") or []:
        for c in cs.get("spec", {}).get("containers", []):
            for e in c.get("env", []):
                env[e["name"]] = e.get("value", "")
    g = pred.get("graph", {})
    env.setdefault("MLOP_MODEL_URI", g.get("modelUri", ""))
    env.setdefault("MLOP_RUNTIME", "mlop-sklearn" if g.get("implementation") == "MLFLOW_SERVER" else "mlop-llm")
    env.setdefault("PREDICTOR_ID", pred.get("name", ""))
    return env


class InProcessLauncher:
    """factory(pod, env) -> backend (blocking build runs in a worker thread)."""

    def __init__(self, factory):
        self.factory = factory

    async def start(self, pod: Pod):
        env = _env_of(pod.spec)
        pod.backend = await asyncio.get_running_loop().run_in_executor(None, self.factory, pod, env)
        pod.ready = True

    async def stop(self, pod: Pod):
        b = pod.backend
        if b is not None and hasattr(b, "stop"):
            b.stop()
        pod.ready = False

    def alive(self, pod: Pod):
        """None = running, else the reason it is gone."""
        b = pod.backend
        return getattr(b, "failure", None) if b is not None else None


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _container_of(pred: dict) -> dict | None:
    for cs in pred.get("componentSpecs") or []:
        for c in cs.get("spec", {}).get("containers", []):
            return c
    return None


class GpuPool:
    """The node's ``amd.com/gpu`` devices as the device plugin hands them out: a pod that asks
    for k GPUs gets k free device indices, exported to its containers as
    ``HIP_VISIBLE_DEVICES`` (so ``cuda:0..k-1`` inside the pod are ITS GPUs and a TP=k
    predictor's ranks land on k distinct GPUs).  ``slots_per_gpu`` > 1 time-shares devices
    (a dev node serving two 8B canary predictors from one MI355X); 1 is the kubelet's
    exclusive assignment.  A request the free slots cannot cover fails like an
    unschedulable pod (``Insufficient amd.com/gpu``)."""

    def __init__(self, devices, slots_per_gpu: int = 1):
        self.devices = list(range(devices)) if isinstance(devices, int) else list(devices)
        self.slots = max(1, int(slots_per_gpu))
        self.used: dict[int, int] = {d: 0 for d in self.devices}

    @classmethod
    def detect(cls, slots_per_gpu: int = 1) -> "GpuPool":
        """Devices visible to this process: HIP_VISIBLE_DEVICES, else the KFD topology in sysfs
        (``rank_launcher.visible_gpu_count``: no HIP / torch call, the launcher of predictor
        processes never touches a GPU itself)."""
        vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
        if vis:
            return cls([int(x) for x in vis.split(",") if x.strip()], slots_per_gpu)
        n = int(os.environ.get("MLOP_NODE_GPUS", "-1"))
        if n < 0:
            from ..runtime.rank_launcher import visible_gpu_count

            n = visible_gpu_count()
        return cls(n, slots_per_gpu)

    @property
    def free(self) -> int:
        return sum(self.slots - u for u in self.used.values())

    def acquire(self, k: int) -> list[int]:
        if k <= 0:
            return []
        # least-used devices first, distinct devices for one pod (its ranks must not share)
        order = sorted((u, d) for d, u in self.used.items() if u < self.slots)
        if len(order) < k:
            raise RuntimeError(f"0/1 nodes are available: Insufficient amd.com/gpu (requested {k}, "
                               f"{len(order)} of {len(self.devices)} devices have a free slot)")
        got = [d for _, d in order[:k]]
        for d in got:
            self.used[d] += 1
        return sorted(got)

    def release(self, devs: list[int]) -> None:
        for d in devs or []:
            if self.used.get(d, 0) > 0:
                self.used[d] -= 1


class ProcessLauncher:
    """One OS process (group) per predictor replica, started from the predictor container's own
    ``command`` / ``args`` as the Seldon controller's pod would (``python`` resolved to this
    interpreter, ``--port`` rewritten to a free local port), with the container env and the
    GPUs the container requests (``amd.com/gpu`` -> ``HIP_VISIBLE_DEVICES`` from ``gpus``, a
    ``GpuPool``).  A TP / EP predictor's container (``--tp N`` / ``--ep N``) launches its own N
    rank processes (runtime/rank_launcher.py).

    ``share_gpu``: the one-GPU node rehearsal of multi-GPU pods.  A pod that asks for k > 1 GPUs
    gets ONE device and ``MLOP_SHARE_GPU=1``, so its N ranks all run on that device over gloo
    with the IPC all-reduce / expert-exchange kernels forced (what ``bench.py --share-gpu``
    does): the operator -> SeldonDeployment -> pod -> launcher -> ranks -> HTTP path runs
    end to end on a box with one MI355X."""

    def __init__(self, scraper=None, extra_env: dict | None = None, python: str = sys.executable,
                 ready_timeout_s: float = 600.0, per_predictor_env: dict | None = None,
                 gpus: GpuPool | int | None = None, gpu_resource: str = "amd.com/gpu", share_gpu: bool = False):
        self.scraper, self.extra_env, self.python = scraper, extra_env or {}, python
        self.share_gpu = share_gpu
        self.per_predictor_env = per_predictor_env or {}  # predictor name -> env (fault injection)
        self.ready_timeout_s = ready_timeout_s
        if gpus is None and self.extra_env.get("MLOP_DEVICE") == "cpu":
            gpus = 8  # CPU emulation of an 8-GPU node: device indices are labels only
        self.gpus = GpuPool(gpus) if isinstance(gpus, int) else (gpus or GpuPool.detect())
        self.gpu_resource = gpu_resource
        # the readiness probe's HTTP client, imported now: a kubelet is a running process, and a
        # first `import aiohttp` (0.15-0.3 s) inside start() would be charged to every CR -> ready
        import aiohttp  # noqa: F401

    def command(self, pod: Pod, port: int) -> list[str]:
        c = _container_of(pod.spec)
        if c is None or not c.get("command"):  # stock MLFLOW_SERVER predictor: our sklearn server
            return [self.python, "-m", "mlopamd.runtime.server", "--port", str(port), "--host", "127.0.0.1"]
        cmd = [self.python if x in ("python", "python3") else x for x in c["command"]]
        args = list(c.get("args") or [])
        for flag, val in (("--port", str(port)), ("--host", "127.0.0.1")):
            if flag in args:
                args[args.index(flag) + 1] = val
            else:
                args += [flag, val]
        return cmd + args

    async def start(self, pod: Pod):
        import aiohttp

        port = free_port()
        env = dict(os.environ)
        env.update(_env_of(pod.spec))
        env.update(self.extra_env)
        env.update(self.per_predictor_env.get(pod.predictor, {}))
        env["SELDON_DEPLOYMENT_ID"] = pod.sd
        env["SELDON_NAMESPACE"] = pod.namespace
        for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT"):  # the pod is its own rank group
            env.pop(k, None)
        need = seldon.gpus_of(pod.spec, self.gpu_resource)
        if self.share_gpu and need > 1:  # rehearsal: the pod's ranks time-share one device
            env["MLOP_SHARE_GPU"] = "1"
            pod.extra["requested_gpus"] = need
            need = 1
        devs = self.gpus.acquire(need)  # raises (unschedulable) when the node has no free GPUs
        pod.extra["gpus"] = devs
        if need:
            env["HIP_VISIBLE_DEVICES"] = ",".join(map(str, devs))
            env.pop("ROCR_VISIBLE_DEVICES", None)
            env.pop("CUDA_VISIBLE_DEVICES", None)
        repo = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = repo + os.pathsep + env.get("PYTHONPATH", "")
        import tempfile

        # stderr to a file: the tail of a dead predictor's log becomes the reason the SD
        # status and the CR report (`kubectl logs --previous` in a real cluster)
        pod.extra["log"] = log_f = tempfile.NamedTemporaryFile(prefix=f"mlop-{pod.predictor}-", suffix=".log",
                                                             delete=False)
        pod.extra["cmd"] = cmd = self.command(pod, port)
        pod.extra["t_start"] = time.perf_counter()
        env["MLOP_LAUNCH_EPOCH"] = repr(time.time())  # the predictor reports its start-up phases against it
        pod.proc = subprocess.Popen(cmd, env=env, stdout=subprocess.DEVNULL,
                                    stderr=log_f, start_new_session=True)
        pod.endpoint = f"http://127.0.0.1:{port}"
        t0 = time.monotonic()
        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=2)) as s:
            while time.monotonic() - t0 < self.ready_timeout_s:
                if pod.proc.poll() is not None:
                    self.gpus.release(pod.extra.pop("gpus", []))
                    raise RuntimeError(f"predictor {pod.predictor} exited with {pod.proc.returncode}: "
                                       f"{self._log_tail(pod)}")
                try:
                    async with s.get(pod.endpoint + "/v2/health/ready") as r:
                        if r.status == 200:
                            pod.ready = True
                            pod.extra["ready_s"] = time.perf_counter() - pod.extra["t_start"]
                            break
                except (aiohttp.ClientError, asyncio.TimeoutError, OSError):
                    pass
                # readiness probe period: 20 ms (a connection refused costs ~0.1 ms, and the
                # probe granularity is part of every measured CR->ready)
                await asyncio.sleep(0.02)
        if self.scraper is not None:
            self.scraper.add_target(pod.endpoint + "/metrics")

    def alive(self, pod: Pod):
        if pod.proc is None or pod.proc.poll() is None:
            return None
        return f"process exited with code {pod.proc.returncode}: {self._log_tail(pod)}"

    @staticmethod
    def _log_tail(pod: Pod, n: int = 240) -> str:
        f = pod.extra.get("log")
        if f is None:
            return ""
        try:
            with open(f.name, "rb") as fh:
                fh.seek(0, 2)
                fh.seek(max(0, fh.tell() - 4096))
                lines = [ln for ln in fh.read().decode("utf-8", "replace").splitlines() if ln.strip()]
            return (lines[-1] if lines else "")[-n:]
        except OSError:
            return ""

    async def stop(self, pod: Pod):
        if self.scraper is not None and pod.endpoint:
            self.scraper.remove_target(pod.endpoint + "/metrics")
        if pod.proc is not None and pod.proc.poll() is None:
            pod.proc.terminate()
            try:
                pod.proc.wait(timeout=20)
            except subprocess.TimeoutExpired:
                # the whole process group: a TP predictor's rank processes included
                try:
                    os.killpg(pod.proc.pid, 9)
                except OSError:
                    pod.proc.kill()
                pod.proc.wait()
        self.gpus.release(pod.extra.pop("gpus", []))
        f = pod.extra.pop("log", None)
        if f is not None:
            f.close()
            try:
                os.unlink(f.name)
            except OSError:
                pass
        pod.ready = False


class SimLauncher:
    """Simulated predictors: every ``period`` (virtual) seconds each ready pod
    records ``rps * period * traffic%`` requests into the MetricStore as the
    Seldon executor would (cumulative histogram buckets, counts per code).
    ``profiles[version] = {"latency": s, "error_rate": f, "startup_s": s}``; an LLM
    predictor profile may add ``tpot`` (s per output token), ``gpu_mem`` (bytes)
    and ``gpu_power`` (W): the runtime's TPOT histogram and amd-smi gauges, and
    ``kernel_shares`` ({class: fraction}): the in-process kernel-time gauge.
    Fault injection: ``fail_start`` (message: the predictor dies while starting, e.g.
    "HIP out of memory"), ``crash_after_s`` (it dies that long after becoming ready;
    ``crashes`` = how many times, default forever: a crash loop)."""

    BUCKETS = (0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0)

    def __init__(self, store, clock, profiles: dict | None = None, rps: float = 50.0, period: float = 5.0):
        self.store, self.clock, self.profiles, self.rps, self.period = store, clock, profiles or {}, rps, period
        self.traffic: dict = {}

    async def start(self, pod: Pod):
        ver = pod.predictor[1:]
        prof = self.profiles.get(ver, {})
        startup = prof.get("startup_s", 0.0)
        if startup:
            await self.clock.sleep(startup)
        if prof.get("fail_start"):
            raise RuntimeError(str(prof["fail_start"]))
        pod.ready = True
        pod.extra["started_at"] = self.clock.now()
        pod.extra.pop("dead", None)
        pod.task = asyncio.get_running_loop().create_task(self._emit(pod, prof))

    def alive(self, pod: Pod):
        prof = self.profiles.get(pod.predictor[1:], {})
        after = prof.get("crash_after_s")
        if pod.extra.get("dead"):
            return pod.extra["dead"]
        if after is not None and pod.ready and pod.restarts < int(prof.get("crashes", 1 << 30)):
            if self.clock.now() - pod.extra.get("started_at", self.clock.now()) >= float(after):
                if pod.task:
                    pod.task.cancel()
                pod.extra["dead"] = "process exited with code 139 (segmentation fault)"
                return pod.extra["dead"]
        return None

    async def _emit(self, pod: Pod, prof: dict):
        lbl = {"deployment_name": pod.sd, "predictor_name": pod.predictor, "namespace": pod.namespace}
        counts = {b: 0.0 for b in self.BUCKETS}
        inf = lsum = ok = err = toks = 0.0
        lat = float(prof.get("latency", 0.05))
        er = float(prof.get("error_rate", 0.0))
        while True:
            share = self.traffic.get(pod.key, 0) / 100.0
            n = self.rps * self.period * share
            if n > 0:
                for b in self.BUCKETS:
                    if lat <= b:
                        counts[b] += n
                inf += n
                lsum += n * lat
                err += n * er
                ok += n * (1 - er)
            t = self.clock.now()
            for b in self.BUCKETS:
                self.store.add("seldon_api_executor_client_requests_seconds_bucket", dict(lbl, le=str(b)), counts[b], t)
            self.store.add("seldon_api_executor_client_requests_seconds_bucket", dict(lbl, le="+Inf"), inf, t)
            self.store.add("seldon_api_executor_client_requests_seconds_sum", lbl, lsum, t)
            self.store.add("seldon_api_executor_client_requests_seconds_count", lbl, inf, t)
            self.store.add("seldon_api_executor_server_requests_seconds_count", dict(lbl, code="200", service="predictions"), ok, t)
            self.store.add("seldon_api_executor_server_requests_seconds_count", dict(lbl, code="500", service="predictions"), err, t)
            if "tpot" in prof:
                toks += n * 32  # 32 output tokens per request
                self.store.add("mlop_time_per_output_token_seconds_sum", lbl, toks * float(prof["tpot"]), t)
                self.store.add("mlop_time_per_output_token_seconds_count", lbl, toks, t)
            if "gpu_mem" in prof:
                self.store.add("mlop_gpu_memory_used_bytes", dict(lbl, gpu="0"), float(prof["gpu_mem"]), t)
            if "gpu_power" in prof:
                self.store.add("mlop_gpu_power_watts", dict(lbl, gpu="0"), float(prof["gpu_power"]), t)
            for k, v in (prof.get("kernel_shares") or {}).items():  # in-process profiler shares
                self.store.add("mlop_kernel_time_fraction", dict(lbl, kernel=k), float(v), t)
            await self.clock.sleep(self.period)

    async def stop(self, pod: Pod):
        if pod.task:
            pod.task.cancel()
        pod.ready = False


class FakeSeldonController:
    """Turns SeldonDeployments into pods and reports their availability."""

    # kubelet-style restart policy: liveness probe period and CrashLoopBackOff (10 s doubling, 300 s cap)
    PROBE_PERIOD_S = 5.0
    BACKOFF_S, BACKOFF_MAX_S = 10.0, 300.0

    def __init__(self, kube, launcher, clock=None):
        self.kube, self.launcher, self.clock = kube, launcher, clock or RealClock()
        self.pods: dict[tuple, Pod] = {}
        self._probe = None
        self.traffic: dict[tuple, int] = {}
        self._task = None
        self._starting: dict[tuple, asyncio.Task] = {}
        self._seen_gen: dict[tuple, int | None] = {}

    def start(self):
        loop = asyncio.get_running_loop()
        self._task = loop.create_task(self._run())
        if hasattr(self.launcher, "alive"):
            self._probe = loop.create_task(self._supervise())
        return self

    async def _supervise(self):
        """Liveness: a predictor that died is reported unavailable (restarts counted in
        the SD status) and restarted after the CrashLoopBackOff delay, like the kubelet
        does for the Seldon pods (restartPolicy Always)."""
        while True:
            await self.clock.sleep(self.PROBE_PERIOD_S)
            for key, pod in list(self.pods.items()):
                if not pod.ready or key in self._starting:
                    continue
                why = self.launcher.alive(pod)
                if why is None:
                    continue
                pod.ready = False
                pod.restarts += 1
                pod.last_error = why
                log.warning("predictor %s/%s/%s died (%s); restart %d", *key, why, pod.restarts)
                await self._report(pod.namespace, pod.sd)
                delay = min(self.BACKOFF_MAX_S, self.BACKOFF_S * 2 ** (pod.restarts - 1))
                self._starting[key] = asyncio.get_running_loop().create_task(self._restart(pod, delay))

    async def _restart(self, pod: Pod, delay: float):
        await self.clock.sleep(delay)
        if self.pods.get(pod.key) is not pod:  # removed meanwhile
            self._starting.pop(pod.key, None)
            return
        try:
            await self.launcher.stop(pod)
        except Exception:  # noqa: BLE001
            pass
        await self._bring_up(pod)

    async def stop(self):
        if self._probe:
            self._probe.cancel()
        if self._task:
            self._task.cancel()
            try:
                await self._task
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass
        for t in self._starting.values():
            t.cancel()
        for pod in list(self.pods.values()):
            await self.launcher.stop(pod)
        self.pods.clear()

    async def _run(self):
        async for etype, sd in self.kube.watch(SELDON_GROUP, SELDON_VERSION, SELDON_PLURAL):
            try:
                await self._reconcile(etype, sd)
            except Exception as e:  # noqa: BLE001
                log.exception("seldon controller: %s", e)

    async def _reconcile(self, etype, sd):
        ns, name = sd["metadata"]["namespace"], sd["metadata"]["name"]
        gen = sd["metadata"].get("generation")
        if etype == "MODIFIED" and self._seen_gen.get((ns, name)) == gen:
            return  # status-only update (our own report): nothing to do
        self._seen_gen[(ns, name)] = None if etype == "DELETED" else gen
        preds = {} if etype == "DELETED" else {p["name"]: p for p in sd["spec"].get("predictors", [])}
        for key in [k for k in self.pods if k[0] == ns and k[1] == name and k[2] not in preds]:
            pod = self.pods.pop(key)
            self.traffic.pop(key, None)
            await self.launcher.stop(pod)
        for pname, p in preds.items():
            key = (ns, name, pname)
            self.traffic[key] = int(p.get("traffic", 0))
            if key not in self.pods:
                pod = Pod(name, ns, pname, p)
                self.pods[key] = pod
                self._starting[key] = asyncio.get_running_loop().create_task(self._bring_up(pod))
        if hasattr(self.launcher, "traffic"):
            self.launcher.traffic = self.traffic
        if etype != "DELETED":
            await self._report(ns, name)

    async def _bring_up(self, pod: Pod):
        try:
            await self.launcher.start(pod)
        except Exception as e:  # noqa: BLE001
            log.error("predictor %s failed to start: %s", pod.predictor, e)
            pod.extra["error"] = str(e)
            pod.last_error = str(e)
        finally:
            self._starting.pop(pod.key, None)
        await self._report(pod.namespace, pod.sd)

    async def _report(self, ns, name):
        mine = {k: p for k, p in self.pods.items() if k[0] == ns and k[1] == name}
        ds = {}
        for (_, _, pname), pod in mine.items():
            g = seldon.graph_name(pname[1:])
            ds[f"{name}-{pname}-0-{g}"] = {"replicas": int(pod.spec.get("replicas", 1)),
                                           "availableReplicas": int(pod.spec.get("replicas", 1)) if pod.ready else 0}
            if pod.restarts or "error" in pod.extra:
                ds[f"{name}-{pname}-0-{g}"].update(restarts=pod.restarts, failed="error" in pod.extra,
                                                   reason=pod.last_error[:300])
        failed = any("error" in p.extra for p in mine.values())
        state = "Failed" if failed else ("Available" if mine and all(p.ready for p in mine.values()) else "Creating")
        try:
            await self.kube.patch_status(SELDON_GROUP, SELDON_VERSION, ns, SELDON_PLURAL, name,
                                         {"status": {"state": state, "deploymentStatus": ds}})
        except ApiError as e:
            if e.status != 404:
                raise

    def backend(self, ns, sd, predictor):
        pod = self.pods.get((ns, sd, predictor))
        return pod.backend if pod else None


class Router:
    """Weighted request routing by the SD traffic split (smooth weighted round-robin)."""

    def __init__(self, controller: FakeSeldonController):
        self.ctl = controller
        self._cw: dict = {}

    def pick(self, ns: str, sd: str) -> Pod | None:
        cands = [(k, w) for k, w in self.ctl.traffic.items() if k[0] == ns and k[1] == sd and w > 0
                 and self.ctl.pods.get(k) is not None and self.ctl.pods[k].ready]
        if not cands:
            return None
        total = sum(w for _, w in cands)
        best = None
        for k, w in cands:
            self._cw[k] = self._cw.get(k, 0) + w
            if best is None or self._cw[k] > self._cw[best]:
                best = k
        self._cw[best] -= total
        return self.ctl.pods[best]

    async def post(self, ns: str, sd: str, path: str, payload: dict, session=None) -> tuple[int, dict, str]:
        import aiohttp

        own = session is None
        session = session or aiohttp.ClientSession()
        try:
            # a predictor removed by a promotion / rollback while a request was in flight
            # resets its connection: retry on a freshly picked pod (the mesh's
            # connect-failure / reset retry policy), 502 when none answers
            for _ in range(3):
                pod = self.pick(ns, sd)
                if pod is None or pod.endpoint is None:
                    return 503, {}, ""
                try:
                    async with session.post(pod.endpoint + path, json=payload) as r:
                        text = await r.text()
                        try:
                            body = json.loads(text) if text else {}
                        except ValueError:  # error responses may be plain text
                            body = {"error": text}
                        return r.status, body, pod.predictor
                except aiohttp.ClientConnectionError as e:
                    last = f"{type(e).__name__}: {e}"
            return 502, {"error": last}, ""
        finally:
            if own:
                await session.close()


def mlflow_model_cr(name: str, namespace: str, model_name: str, alias: str, interval: int = 60,
                    secret: str | None = "minio-secret", **extra_spec) -> dict:
    spec = {"modelName": model_name, "modelAlias": alias, "monitoringInterval": interval}
    if secret:
        spec["minioSecret"] = secret
    spec.update(extra_spec)
    return {"apiVersion": API_VERSION, "kind": KIND, "metadata": {"name": name, "namespace": namespace},
            "spec": spec}


async def wait_for(pred, timeout_s: float = 60.0, poll_s: float = 0.01):
    t0 = time.monotonic()
    while time.monotonic() - t0 < timeout_s:
        v = await pred()
        if v:
            return v
        await asyncio.sleep(poll_s)
    raise TimeoutError("condition not met")


# ---------------------------------------------------------------- bench --

def deploy_and_wait(model: str = "llama3-8b", device="cuda", seed: int = 0, engine_kwargs: dict | None = None,
                    namespace: str = "serving", timeout_s: float = 900.0):
    """Run the full control-plane path in-process: MLflow registry (sqlite) holds
    the model version with its architecture tag, an MlflowModel CR is created,
    the operator reconciles it into a SeldonDeployment whose predictor is our
    LLM runtime, the fake Seldon controller brings that predictor up on THIS
    process's GPU, and the CR reports ready.  Returns (engine, info)."""
    from ..runtime.deploy import build_engine
    from .app import OperatorMetrics, make_operator
    from .crd import OperatorSettings
    from .mlflow import LocalMlflowClient, SqliteRegistry
    from .prometheus import LocalProm, MetricStore

    engine_kwargs = dict(engine_kwargs or {})

    async def main():
        kube = FakeKube()
        reg = SqliteRegistry()
        reg.create_model_version(model, f"mlflow-artifacts:/1/{model}/artifacts/model",
                                 tags={"mlop.architecture": model, "mlop.runtime": seldon.RUNTIME_LLM})
        reg.set_alias(model, "champion", 1)
        clock = RealClock()
        metrics = OperatorMetrics()
        op, rec = make_operator(kube, LocalMlflowClient(reg), LocalProm(MetricStore()), clock,
                                OperatorSettings(), metrics=metrics)
        built = {}

        def factory(pod, env):
            import torch

            if torch.device(device).type == "cuda":
                torch.cuda.set_device(device)  # worker thread: HIP's current device is per-thread
            eng = build_engine(env.get("MLOP_ARCHITECTURE", model), device=device, seed=seed,
                               model_uri=env.get("MLOP_MODEL_URI"), **engine_kwargs)
            built["engine"] = eng
            return eng

        ctl = FakeSeldonController(kube, InProcessLauncher(factory), clock).start()
        await op.start()
        t0 = time.perf_counter()
        cr = mlflow_model_cr(model, namespace, model, "champion", interval=60,
                             maxNumSeqs=engine_kwargs.get("max_num_seqs", 256),
                             maxModelLen=engine_kwargs.get("max_model_len", 4096))
        await kube.create(GROUP, VERSION, namespace, PLURAL, cr)

        async def ready():
            o = await kube.get(GROUP, VERSION, namespace, PLURAL, model)
            if (o.get("status") or {}).get("ready") == "True":
                return o
            # a predictor that cannot start (e.g. GPU OOM at weight load) fails the deploy
            # now instead of at the timeout
            try:
                sd = await kube.get(SELDON_GROUP, SELDON_VERSION, namespace, SELDON_PLURAL, model)
            except ApiError:
                return False
            for p in sd["spec"]["predictors"]:
                _, failed, reason = seldon.predictor_health(sd, p["name"])
                if failed:
                    raise RuntimeError(f"predictor {p['name']} failed to start: {reason}")
            return False

        obj = await wait_for(ready, timeout_s)
        ready_s = time.perf_counter() - t0
        sd = await kube.get(SELDON_GROUP, SELDON_VERSION, namespace, SELDON_PLURAL, model)
        pred = sd["spec"]["predictors"][0]
        info = {"cr_ready_s": round(ready_s, 3), "phase": obj["status"].get("phase"),
                "predictor": pred["name"], "runtime": pred.get("annotations", {}).get("mlop.amd.com/runtime"),
                "placement": {k.split("/")[-1]: v for k, v in pred.get("annotations", {}).items()
                              if k != "mlop.amd.com/runtime"},
                "events": [e["reason"] for e in kube.events],
                "weight_gb": round(built["engine"].model.weight_bytes() / 1e9, 2),
                "kv_blocks": built["engine"].kv.num_blocks}
        # hand the engine to the caller: stop the control loops, keep the engine
        ctl.pods.clear()
        await ctl.stop()
        await op.stop()
        return built["engine"], info

    return asyncio.run(main())
