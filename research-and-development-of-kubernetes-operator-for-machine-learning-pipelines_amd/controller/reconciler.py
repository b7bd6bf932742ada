"""MlflowModel reconciler: alias polling, deployment, canary, rollback (reference C4/C5/C8).

One daemon per CR (framework.Operator) runs ``MlflowModelReconciler.run``:

  every tick (<= monitoringInterval):
    alias -> version           (MLflow; NotFound vs RegistryUnavailable, C5 fixed)
    new version?  -> status {current, previous, error: null, phase}, Event NewModelVersionDetected
    desired SD from STATUS      (level-triggered: re-applied whenever the live SD differs)
    readiness of the current predictor -> status.ready / readyTime, Event PredictorReady
    canary (phase Canary) advances by persisted timestamps, never blocking the poll

Canary schedule (reference mlflow_operator.py:175-179,184-191,288-361): start
at initialTraffic (10) for the new predictor; every ``interval`` after a
passing gate +step (10); failed gate attempts every ``attemptDelay`` (10 s);
after ``maxAttempts`` (10) failures -> Event PromotionFailed and — new — a
real rollback (previous version back to 100 %, the new predictor removed,
``status.rolledBackVersion`` set so the same alias version is not redeployed
in a loop).  At 100 % the old predictor is removed (Event PromotionComplete).
The gate starts only once the new predictor is READY (reference gated
immediately; LLM predictors need minutes to load).  All canary progress lives
in the CR status, so an operator restart resumes mid-canary.
"""
from __future__ import annotations

import asyncio
import logging

from . import seldon
from .crd import (EV_ALIAS_NOT_FOUND, EV_NEW_VERSION, EV_PREDICTOR_READY, EV_PREDICTOR_UNAVAILABLE,
                  EV_METRICS_UNAVAILABLE, EV_PROMOTION_COMPLETE, EV_PROMOTION_FAILED, EV_REGISTRY_UNAVAILABLE, EV_ROLLBACK_COMPLETE,
                  EV_TRAFFIC_INCREASE, GROUP, PLURAL, SELDON_GROUP, SELDON_PLURAL, SELDON_VERSION,
                  VERSION, ModelSpec, OperatorSettings, artifact_uri)
from .kube import ApiError
from .mlflow import NotFound, RegistryError, RegistryUnavailable
from .placement import plan

from .prometheus import MetricsUnavailable, get_model_metrics, gpu_guard_queries, should_promote

ANN = seldon.ANN_PREFIX
SELDON_POD_LABEL = seldon.POD_LABEL

PH_DEPLOYING, PH_READY, PH_CANARY = "Deploying", "Ready", "Canary"
PH_PROMOTED, PH_ROLLED_BACK, PH_FAILED, PH_NO_ALIAS = "Promoted", "RolledBack", "PromotionFailed", "AliasNotFound"


class MlflowModelReconciler:
    def __init__(self, kube, mlflow, prom, clock, operator, settings: OperatorSettings | None = None,
                 metrics=None):
        self.kube, self.mlflow, self.prom, self.clock, self.op = kube, mlflow, prom, clock, operator
        self.settings = settings or OperatorSettings()
        self.metrics = metrics  # optional OperatorMetrics (reconcile latency, CR->ready)
        self._kicks = {}
        self.placement_notes: dict = {}  # (ns, name) -> {predictor: why it cannot be placed}

    # ------------------------------------------------------------- k8s --
    async def _get_cr(self, ns, name):
        return await self.kube.get(GROUP, VERSION, ns, PLURAL, name)

    async def _patch_status(self, ns, name, patch: dict):
        return await self.kube.patch_status(GROUP, VERSION, ns, PLURAL, name, {"status": patch})

    async def _get_sd(self, ns, name):
        try:
            return await self.kube.get(SELDON_GROUP, SELDON_VERSION, ns, SELDON_PLURAL, name)
        except ApiError as e:
            if e.status == 404:
                return None
            raise

    async def apply_sd(self, desired: dict, logger) -> dict:
        """Idempotent apply (reference C7) with optimistic-concurrency retry on 409
        (the reference re-raised it, mlflow_operator.py:280-282)."""
        md = desired["metadata"]
        ns, name = md["namespace"], md["name"]
        for attempt in range(5):
            cur = await self._get_sd(ns, name)
            try:
                if cur is None:
                    return await self.kube.create(SELDON_GROUP, SELDON_VERSION, ns, SELDON_PLURAL, desired)
                if seldon.spec_equal(cur, desired) and cur["metadata"].get("ownerReferences") == md.get("ownerReferences"):
                    return cur
                body = dict(desired)
                body["metadata"] = dict(md, resourceVersion=cur["metadata"]["resourceVersion"])
                return await self.kube.replace(SELDON_GROUP, SELDON_VERSION, ns, SELDON_PLURAL, name, body)
            except ApiError as e:
                if e.status in (409,) and attempt < 4:
                    logger.info("[%s/%s] SeldonDeployment conflict, retrying with a fresh resourceVersion", ns, name)
                    continue
                logger.error("[%s/%s] Error applying SeldonDeployment: %s", ns, name, e)
                raise
        raise ApiError(409, "Conflict", "gave up after 5 conflicting writes")

    async def delete_sd(self, ns, name, logger):
        """Reference C10: delete, ignore 404, re-raise the rest."""
        try:
            await self.kube.delete(SELDON_GROUP, SELDON_VERSION, ns, SELDON_PLURAL, name)
            logger.info("[%s/%s] SeldonDeployment '%s' deleted from namespace '%s'.", ns, name, name, ns)
        except ApiError as e:
            if e.status != 404:
                logger.error("[%s/%s] Error deleting SeldonDeployment '%s': %s", ns, name, name, e)
                raise

    # ------------------------------------------------------------ nodes --
    async def node_capacity(self, exclude: tuple | None = None) -> dict:
        """The GPU node a new predictor would land on, as the scheduler sees it: Node objects'
        ``status.allocatable[amd.com/gpu]`` (the device plugin's count) and HBM per GPU from
        the AMD node labeller's ``amd.com/gpu.vram`` label (e.g. ``288G``), minus the GPUs
        other SeldonDeployments' predictors already request (replicas x limits).  Picks the
        node with the most free GPUs.  {} when no node exposes the resource (or nodes cannot
        be listed): the planner then uses the operator settings (RBAC
        ``nodes`` get/list/watch, manifests/rbac.yaml)."""
        res = self.settings.gpu_resource
        try:
            nodes = await self.kube.list("", "v1", None, "nodes")
        except Exception:  # noqa: BLE001 - no RBAC / no node API: static settings
            return {}
        cands = []
        for n in nodes:
            alloc = ((n.get("status") or {}).get("allocatable") or {}).get(res)
            if not alloc:
                continue
            labels = (n.get("metadata") or {}).get("labels") or {}
            vram = labels.get(f"{res}.vram") or labels.get("amd.com/gpu.vram")
            hbm = None
            if vram:
                try:
                    hbm = float(str(vram).rstrip("GgBi"))
                except ValueError:
                    hbm = None
            cands.append({"node": n["metadata"]["name"], "gpus": int(alloc), "hbm_gb": hbm})
        if not cands:
            return {}
        # per-node accounting from the pods bound to each node (GPU limits of pods that still
        # hold their devices); without pod access, the SeldonDeployments' total is charged to
        # the cluster and the roomiest node reports min(its GPUs, the cluster's free GPUs)
        per_node = await self._gpus_used_per_node(res, exclude)
        if per_node is not None:
            for c in cands:
                c["free"] = max(0, c["gpus"] - per_node.get(c["node"], 0))
            best = max(cands, key=lambda c: (c["free"], c["gpus"]))
            out = {"node": best["node"], "gpus": best["gpus"], "free_gpus": best["free"], "accounting": "per-node"}
        else:
            used = 0
            try:
                sds = await self.kube.list(SELDON_GROUP, SELDON_VERSION, None, SELDON_PLURAL)
            except Exception:  # noqa: BLE001
                sds = []
            for sd in sds:
                md = sd.get("metadata") or {}
                if exclude and (md.get("namespace"), md.get("name")) == exclude:
                    continue
                for p in (sd.get("spec") or {}).get("predictors", []):
                    used += int(p.get("replicas", 1)) * seldon.gpus_of(p, res)
            best = max(cands, key=lambda c: c["gpus"])
            cluster_free = max(0, sum(c["gpus"] for c in cands) - used)
            out = {"node": best["node"], "gpus": best["gpus"], "free_gpus": min(best["gpus"], cluster_free),
                   "accounting": "cluster (pods not listable: requests charged cluster-wide)"}
        if best["hbm_gb"]:
            out["hbm_gb"] = best["hbm_gb"]
        return out

    async def _gpus_used_per_node(self, res: str, exclude: tuple | None = None) -> dict | None:
        """{node: GPUs requested by the pods bound to it and not finished}, or None when pods
        cannot be listed (no RBAC / no pod API in this cluster emulation).  ``exclude`` =
        (namespace, SeldonDeployment name): that deployment's OWN predictor pods (Seldon v1
        labels every pod it creates ``seldon-deployment-id: <SD name>``) are not charged, so
        the model's running predictors never count against its own re-planned placement."""
        try:
            pods = await self.kube.list("", "v1", None, "pods")
        except Exception:  # noqa: BLE001
            return None
        if not pods:
            return None
        used: dict = {}
        for pod in pods:
            spec, st = pod.get("spec") or {}, pod.get("status") or {}
            node = spec.get("nodeName")
            if not node or st.get("phase") in ("Succeeded", "Failed"):
                continue
            pmd = pod.get("metadata") or {}
            if exclude and (pmd.get("namespace"), (pmd.get("labels") or {}).get(SELDON_POD_LABEL)) == exclude:
                continue
            n = 0
            for c in spec.get("containers") or []:
                lim = ((c.get("resources") or {}).get("limits") or {}).get(res)
                if lim:
                    n += int(lim)
            used[node] = used.get(node, 0) + n
        return used

    # --------------------------------------------------------- desired --
    async def _uri(self, spec: ModelSpec, version) -> tuple[str, object]:
        mv = await self.mlflow.get_model_version(spec.model_name, version)
        return artifact_uri(mv.source, self.settings.artifact_base), mv

    def _runtime_of(self, spec: ModelSpec, mv) -> tuple[str, str | None]:
        tags = getattr(mv, "tags", {}) or {}
        arch = spec.architecture or tags.get("mlop.architecture")
        rt = spec.runtime or tags.get("mlop.runtime") or (seldon.RUNTIME_LLM if arch else seldon.RUNTIME_STOCK)
        return rt, arch

    @staticmethod
    def _placement_key(spec: ModelSpec, arch: str) -> str:
        """Everything a version's placement is planned from, besides the cluster's momentary
        free capacity: a deployed predictor keeps its placement while this key is unchanged."""
        return (f"{arch}|tp={spec.tensor_parallel or 0}|ep={spec.expert_parallel or 0}"
                f"|len={spec.max_model_len or 4096}|seqs={spec.max_num_seqs or 256}"
                f"|kvf={spec.kv_target_fraction or 0.5}|replicas={spec.replicas}")

    async def desired_sd(self, body: dict, spec: ModelSpec, status: dict) -> dict | None:
        """The SeldonDeployment this CR wants now.  Placement is decided ONCE per version, like
        a scheduled pod that does not move: a predictor already deployed with a placement that
        fit, planned from the same inputs (``_placement_key``), keeps it — so level-triggered
        reconciles never rewrite the SD spec because GPU counts moved (its own pods, a rollout).
        Only the stable plan goes into the predictor annotations; the planner's reason text,
        which quotes momentary free counts, goes to the CR status (``placement``)."""
        md = body["metadata"]
        cur, prev = status.get("currentModelVersion"), status.get("previousModelVersion")
        if cur is None:
            return None
        phase = status.get("phase")
        preds = []
        # PromotionFailed without rollback keeps the split the canary stopped at (reference
        # mlflow_operator.py:347-349 leaves it); only Canary and PromotionFailed carry two predictors
        split = phase in (PH_CANARY, PH_FAILED) and prev is not None
        ct = int(status.get("canaryTraffic") or 0)
        versions = [(prev, 100 - ct), (cur, ct)] if split else [(cur, 100)]
        node = None
        existing = None
        notes = {}
        # GPUs of this SD's predictors placed earlier in this pass while no node had been read
        # yet (a reused placement skips the node read).  node_capacity excludes the SD's OWN
        # pods, so a later predictor's free count must be charged with them explicitly: a canary
        # never plans onto the GPUs the running version still holds
        held_before_node = 0
        for v, traffic in versions:
            uri, mv = await self._uri(spec, v)
            runtime, arch = self._runtime_of(spec, mv)
            placement = None
            if runtime == seldon.RUNTIME_LLM and arch:
                if existing is None:
                    existing = {p["name"]: p for p in ((await self._get_sd(md["namespace"], md["name"])) or {})
                                .get("spec", {}).get("predictors", [])}
                key = self._placement_key(spec, arch)
                ann = (existing.get(seldon.predictor_name(v)) or {}).get("annotations") or {}
                if ann.get(f"{ANN}placementKey") == key and ann.get(f"{ANN}fits") == "True":
                    placement = {k[len(ANN):]: val for k, val in ann.items()
                                 if k.startswith(ANN) and k != f"{ANN}runtime"}
                    gpus_held = int(placement.get("gpus", 0))
                else:
                    if node is None:
                        node = await self.node_capacity(exclude=(md["namespace"], md["name"]))
                        if node.get("free_gpus") is not None and held_before_node:
                            node = dict(node, free_gpus=max(0, node["free_gpus"] - held_before_node))
                    p = plan(arch, max_model_len=spec.max_model_len or 4096, max_num_seqs=spec.max_num_seqs or 256,
                             hbm_gb=node.get("hbm_gb", self.settings.hbm_per_gpu_gb),
                             gpus_per_node=node.get("gpus", self.settings.gpus_per_node),
                             requested_tp=spec.tensor_parallel, requested_ep=spec.expert_parallel,
                             kv_target_fraction=spec.kv_target_fraction or 0.5,
                             free_gpus=node.get("free_gpus"))
                    placement = {"tensorParallel": p.tensorParallel, "expertParallel": p.expertParallel,
                                 "gpus": p.gpus, "weightGBPerGPU": p.weightGBPerGPU,
                                 "kvTokenCapacity": p.kvTokenCapacity, "fits": p.fits, "placementKey": key}
                    if node.get("node"):
                        placement["node"] = node["node"]
                    if not p.fits:
                        notes[seldon.predictor_name(v)] = p.reason + (
                            f" [GPU accounting: {node['accounting']}]" if node.get("accounting") else "")
                    gpus_held = p.gpus
                if node is None:
                    held_before_node += gpus_held * spec.replicas
                elif node.get("free_gpus") is not None:
                    # the canary's second predictor needs its own GPUs beside this one's
                    node = dict(node, free_gpus=max(0, node["free_gpus"] - gpus_held * spec.replicas))
            elif runtime == seldon.RUNTIME_LLM and (spec.tensor_parallel or spec.expert_parallel):
                # a checkpoint of unknown architecture (no preset): honour the requested degrees
                tp = int(spec.tensor_parallel or 1)
                ep = int(spec.expert_parallel or 1)
                placement = {"tensorParallel": tp, "expertParallel": ep, "gpus": max(tp, ep)}
            engine_args = {}
            if spec.max_model_len:
                engine_args["max_model_len"] = spec.max_model_len
            if spec.max_num_seqs:
                engine_args["max_num_seqs"] = spec.max_num_seqs
            preds.append(seldon.build_predictor(
                v, uri, spec.minio_secret, traffic, runtime=runtime, replicas=spec.replicas, placement=placement,
                image=self.settings.runtime_image, gpu_resource=self.settings.gpu_resource,
                model_name=spec.model_name, deployment=md["name"], namespace=md["namespace"],
                architecture=arch, engine_args=engine_args))
        self.placement_notes[(md["namespace"], md["name"])] = notes
        return seldon.build_seldon_deployment(md["name"], md["namespace"], body, preds)

    # -------------------------------------------------------------- run --
    async def run(self, body: dict, stopped: asyncio.Event, logger: logging.Logger | None = None):
        md = body["metadata"]
        ns, name = md["namespace"], md["name"]
        logger = logger or logging.getLogger(f"{name}-{ns}")
        spec = ModelSpec.from_spec(body.get("spec"))
        errs = spec.validate()
        if errs:
            await self._patch_status(ns, name, {"error": "; ".join(errs), "phase": "Invalid"})
            logger.error("[%s/%s] invalid spec: %s", ns, name, errs)
            return
        kick = self._kicks.setdefault((ns, name), asyncio.Event())
        try:
            while not stopped.is_set():
                kick.clear()
                try:
                    wait = await self.tick(ns, name, spec, logger)
                except ApiError as e:
                    if e.status == 404:  # CR deleted (reference crashed here)
                        return
                    logger.warning("[%s/%s] reconcile error: %s", ns, name, e)
                    wait = min(spec.monitoring_interval, 10.0)
                except asyncio.CancelledError:
                    raise
                except Exception:  # noqa: BLE001 - any other failure retries (kopf's handler
                    # retry); it must not end this CR's daemon for good
                    logger.exception("[%s/%s] unexpected reconcile error; retrying", ns, name)
                    wait = min(spec.monitoring_interval, 10.0)
                await self._sleep_or_kick(wait, kick)
        finally:
            self._kicks.pop((ns, name), None)

    _kicks: dict = {}

    def kick(self, ns: str, name: str):
        """Wake a CR's loop now (an owned SeldonDeployment changed, e.g. became ready)."""
        ev = self._kicks.get((ns, name))
        if ev is not None:
            ev.set()

    async def _sleep_or_kick(self, seconds: float, kick: asyncio.Event):
        sl = asyncio.ensure_future(self.clock.sleep(seconds))
        kw = asyncio.ensure_future(kick.wait())
        try:
            await asyncio.wait({sl, kw}, return_when=asyncio.FIRST_COMPLETED)
        finally:
            for t in (sl, kw):
                if not t.done():
                    t.cancel()

    async def tick(self, ns, name, spec: ModelSpec, logger) -> float:
        """One reconcile pass; returns seconds until the next one."""
        t0 = self.clock.monotonic()
        body = await self._get_cr(ns, name)
        status = dict(body.get("status") or {})
        interval = spec.monitoring_interval
        # ---- alias lookup
        try:
            mv = await self.mlflow.get_model_version_by_alias(spec.model_name, spec.model_alias)
        except NotFound:
            if status.get("phase") != PH_NO_ALIAS:
                await self._patch_status(ns, name, {"error": f"Alias '{spec.model_alias}' does not exist",
                                                    "currentModelVersion": None, "previousModelVersion": None,
                                                    "phase": PH_NO_ALIAS, "ready": "False", "canaryTraffic": None})
                await self.delete_sd(ns, name, logger)
                await self.op.event(body, "Warning", EV_ALIAS_NOT_FOUND,
                                    f"Alias '{spec.model_alias}' does not exist.")
            logger.error("[%s/%s] Alias '%s' does not exist.", ns, name, spec.model_alias)
            return interval
        except (RegistryUnavailable, RegistryError) as e:
            # transient: keep serving what is deployed (the reference deleted it)
            if status.get("registryUnavailable") != "True":
                await self._patch_status(ns, name, {"registryUnavailable": "True"})
                await self.op.event(body, "Warning", EV_REGISTRY_UNAVAILABLE, f"MLflow registry unavailable: {e}")
            logger.warning("[%s/%s] registry unavailable (%s); keeping the current deployment", ns, name, e)
            return min(interval, 15.0)
        if status.get("registryUnavailable") == "True":
            await self._patch_status(ns, name, {"registryUnavailable": None})
        new = str(mv.version)
        cur = status.get("currentModelVersion")
        now = self.clock.now()

        if new != cur and new == status.get("rolledBackVersion"):
            pass  # anti-flap: this version failed its canary; wait for a different alias target
        elif new != cur:
            sd = await self._get_sd(ns, name)
            serving = seldon.traffic_of(sd)
            prev = cur if (cur is not None and serving.get(seldon.predictor_name(cur), 0) > 0) else None
            if status.get("phase") in (PH_CANARY, PH_FAILED) and prev is not None:
                # a newer version arrived mid-canary (or after a failed one left its split):
                # keep the one with the most traffic as the baseline
                old_prev = status.get("previousModelVersion")
                if old_prev is not None and serving.get(seldon.predictor_name(old_prev), 0) >= serving.get(
                        seldon.predictor_name(cur), 0):
                    prev = old_prev
            patch = {"currentModelVersion": new, "previousModelVersion": prev, "error": None,
                     "phase": PH_CANARY if prev is not None else PH_DEPLOYING,
                     "canaryTraffic": spec.canary.initial_traffic if prev is not None else 100,
                     "canaryStepStarted": now, "canaryNextAttempt": now, "canaryAttempts": 0,
                     "ready": "False", "readyTime": None, "versionDetectedTime": now,
                     "rolledBackVersion": None}
            body = await self._patch_status(ns, name, patch)
            status.update(patch)
            logger.info("[%s/%s] New model version detected: %s", ns, name, new)
            await self.op.event(body, "Normal", EV_NEW_VERSION, f"New model version {new} detected.")

        # ---- level-triggered apply of the desired deployment
        desired = await self.desired_sd(body, spec, status)
        notes = self.placement_notes.pop((ns, name), None) or None  # consumed: no stale entries
        if desired is not None and status.get("placement") != notes:  # why a predictor cannot be placed
            body = await self._patch_status(ns, name, {"placement": notes})
            status["placement"] = notes
        if desired is not None:
            sd = await self.apply_sd(desired, logger)
        else:
            sd = await self._get_sd(ns, name)
        # ---- readiness of the current predictor
        cur = status.get("currentModelVersion")
        pcur = seldon.predictor_name(cur)
        cur_ready = cur is not None and seldon.predictor_ready(sd, pcur)
        if cur is not None and status.get("ready") != "True" and cur_ready:
            created = body["metadata"].get("creationTimestamp")
            first = status.get("readyTime") is None
            ready_patch = {"ready": "True", "readyTime": now if first else status.get("readyTime")}
            if status.get("phase") == PH_DEPLOYING:
                ready_patch["phase"] = PH_READY
            body = await self._patch_status(ns, name, ready_patch)
            status.update(ready_patch)
            dt = now - float(status.get("versionDetectedTime") or now)
            if first and self.metrics:
                self.metrics.observe_ready(dt)
            await self.op.event(body, "Normal", EV_PREDICTOR_READY,
                                f"Predictor {pcur} ready {dt:.1f}s after version detection (CR created {created})."
                                if first else f"Predictor {pcur} available again after a restart.")
        elif cur is not None and status.get("ready") == "True" and sd is not None and not cur_ready:
            # the serving predictor died (crash, GPU fault): the Seldon controller restarts
            # it; surface the outage on the CR until it is back
            restarts, _, reason = seldon.predictor_health(sd, pcur)
            body = await self._patch_status(ns, name, {"ready": "False", "predictorRestarts": restarts})
            status.update(ready="False", predictorRestarts=restarts)
            await self.op.event(body, "Warning", EV_PREDICTOR_UNAVAILABLE,
                                f"Predictor {pcur} unavailable (restart {restarts}): {reason}"[:1000])
        wait = interval
        if status.get("phase") == PH_CANARY:
            wait = min(wait, await self.canary_tick(body, ns, name, spec, status, sd, logger))
        if self.metrics:
            self.metrics.observe_reconcile(self.clock.monotonic() - t0)
        return max(0.01, wait)

    # ----------------------------------------------------------- canary --
    async def canary_tick(self, body, ns, name, spec: ModelSpec, status: dict, sd, logger) -> float:
        pol = spec.canary
        now = self.clock.now()
        cur, prev = status["currentModelVersion"], status.get("previousModelVersion")
        pc, pp = seldon.predictor_name(cur), seldon.predictor_name(prev)
        restarts, failed, reason = seldon.predictor_health(sd, pc)
        if failed or restarts >= pol.max_restarts:
            # a canary that cannot start (GPU OOM at load) or crash-loops never gets
            # healthy: fail it now instead of after ready_timeout (SURVEY.md §5 recovery)
            why = (f"new predictor {pc} failed to start: {reason}" if failed else
                   f"new predictor {pc} restarted {restarts} times: {reason}")
            logger.warning("[%s/%s] %s", ns, name, why)
            await self._fail(body, ns, name, spec, status, logger, why, unhealthy=True)
            return 0.01
        if not seldon.predictor_ready(sd, pc):
            if now - float(status.get("canaryStepStarted", now)) > pol.ready_timeout_s:
                logger.warning("[%s/%s] new predictor %s not ready after %.0fs", ns, name, pc, pol.ready_timeout_s)
                await self._fail(body, ns, name, spec, status, logger, "new predictor never became ready",
                                 unhealthy=True)
                return 0.01
            return min(5.0, pol.attempt_delay_s)
        next_at = float(status.get("canaryNextAttempt", now))
        if now < next_at:
            return next_at - now
        guards = pol.gpu_guards or {}
        try:
            new_m = await get_model_metrics(self.prom, name, pc, ns, pol.window_s,
                                            extra_queries=guards and gpu_guard_queries(name, pc, ns, pol.window_s))
            old_m = await get_model_metrics(self.prom, name, pp, ns, pol.window_s,
                                            extra_queries=guards and gpu_guard_queries(name, pp, ns, pol.window_s))
        except MetricsUnavailable as e:
            # the metrics backend is down: hold the split, do not count an attempt (the
            # reference's sync client raised here and its handler died mid-canary)
            if status.get("metricsUnavailable") != "True":
                status["metricsUnavailable"] = "True"
                body = await self._patch_status(ns, name, {"metricsUnavailable": "True"})
                logger.warning("[%s/%s] metrics backend unavailable, canary paused: %s", ns, name, e)
                await self.op.event(body, "Warning", EV_METRICS_UNAVAILABLE,
                                    f"Prometheus unavailable, canary paused at {status.get('canaryTraffic')}%: {e}"[:1000])
            return pol.attempt_delay_s
        if status.get("metricsUnavailable") == "True":
            status["metricsUnavailable"] = None
            await self._patch_status(ns, name, {"metricsUnavailable": None})
        logger.info("[%s/%s] Metrics for new model (version %s): %s", ns, name, cur, new_m)
        logger.info("[%s/%s] Metrics for old model (version %s): %s", ns, name, prev, old_m)
        gate = should_promote(new_m, old_m, pol.thresholds, pol.error_rate_floor, logger=logger,
                              latency_floor_s=pol.latency_floor_s, extra_max_ratio=guards)
        if gate.promote:
            traffic = min(100, int(status.get("canaryTraffic", 0)) + pol.step)
            if traffic >= 100:
                patch = {"phase": PH_PROMOTED, "canaryTraffic": 100, "canaryAttempts": 0}
                body = await self._patch_status(ns, name, patch)
                status.update(patch)
                await self.apply_sd(await self.desired_sd(body, spec, status), logger)
                logger.info("[%s/%s] The new model has received 100%% of traffic. Previous model has been removed.", ns, name)
                await self.op.event(body, "Normal", EV_PROMOTION_COMPLETE,
                                    "New model now receives 100% traffic. Previous model has been removed.")
                return spec.monitoring_interval
            patch = {"canaryTraffic": traffic, "canaryAttempts": 0, "canaryStepStarted": now,
                     "canaryNextAttempt": now + pol.interval_s}
            body = await self._patch_status(ns, name, patch)
            status.update(patch)
            await self.apply_sd(await self.desired_sd(body, spec, status), logger)
            logger.info("[%s/%s] Increased traffic to new model to %d%%", ns, name, traffic)
            await self.op.event(body, "Normal", EV_TRAFFIC_INCREASE, f"Increased traffic to new model to {traffic}%")
            return pol.interval_s
        attempts = int(status.get("canaryAttempts", 0)) + 1
        if attempts < pol.max_attempts:
            patch = {"canaryAttempts": attempts, "canaryNextAttempt": now + pol.attempt_delay_s,
                     "canaryLastGate": "; ".join(gate.reasons)[:500]}
            await self._patch_status(ns, name, patch)
            logger.info("[%s/%s] Attempt %d/%d: Metrics do not meet conditions, retrying after %.0f seconds.",
                        ns, name, attempts, pol.max_attempts, pol.attempt_delay_s)
            return pol.attempt_delay_s
        await self._fail(body, ns, name, spec, status, logger, "; ".join(gate.reasons))
        return 0.01

    async def _fail(self, body, ns, name, spec, status, logger, why: str, unhealthy: bool = False):
        pol = spec.canary
        if unhealthy:  # the canary predictor itself failed (start error, crash loop, never ready)
            msg = f"Canary predictor unhealthy ({why}), stopping promotion."
        else:  # the reference's message (mlflow_operator.py:343-344)
            msg = f"Metrics did not meet conditions after {pol.max_attempts} attempts, stopping promotion."
        logger.warning("[%s/%s] %s", ns, name, msg)
        await self.op.event(body, "Warning", EV_PROMOTION_FAILED, msg[:1000])
        if not pol.rollback:  # reference behaviour: leave the split as it is
            await self._patch_status(ns, name, {"phase": PH_FAILED, "canaryLastGate": why[:500]})
            return
        failed, prev = status["currentModelVersion"], status.get("previousModelVersion")
        patch = {"phase": PH_ROLLED_BACK, "currentModelVersion": prev, "previousModelVersion": None,
                 "rolledBackVersion": failed, "canaryTraffic": 100, "ready": "True",
                 "error": f"version {failed} rolled back: {why}"[:500]}
        body = await self._patch_status(ns, name, patch)
        status.update(patch)
        await self.apply_sd(await self.desired_sd(body, spec, status), logger)
        logger.warning("[%s/%s] Rolled back to version %s (version %s failed its canary)", ns, name, prev, failed)
        await self.op.event(body, "Warning", EV_ROLLBACK_COMPLETE,
                            f"Rolled back to version {prev}; version {failed} failed its canary: {why}"[:1000])
