"""MlflowModel resource contract (reference crd.yaml:1-46) and operator settings.

Spec fields (reference): modelName, modelAlias, monitoringInterval (default
60 s, mlflow_operator.py:31), minioSecret.  Status fields (reference):
currentModelVersion, previousModelVersion, error.  Everything else here is
an optional extension with a default that reproduces the reference behaviour.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from pathlib import Path

import yaml

GROUP = "mlflow.nizepart.com"
VERSION = "v1alpha1"
PLURAL = "mlflowmodels"
KIND = "MlflowModel"
API_VERSION = f"{GROUP}/{VERSION}"

SELDON_GROUP = "machinelearning.seldon.io"
SELDON_VERSION = "v1"
SELDON_PLURAL = "seldondeployments"
SELDON_KIND = "SeldonDeployment"

MANIFESTS = Path(__file__).resolve().parents[2] / "manifests"

# K8s Event reasons: the reference's five (mlflow_operator.py:90,122,332,344,361) + ours
EV_ALIAS_NOT_FOUND = "AliasNotFound"
EV_NEW_VERSION = "NewModelVersionDetected"
EV_TRAFFIC_INCREASE = "TrafficIncrease"
EV_PROMOTION_FAILED = "PromotionFailed"
EV_PROMOTION_COMPLETE = "PromotionComplete"
EV_ROLLBACK_COMPLETE = "RollbackComplete"
EV_PREDICTOR_READY = "PredictorReady"
EV_PREDICTOR_UNAVAILABLE = "PredictorUnavailable"
EV_REGISTRY_UNAVAILABLE = "RegistryUnavailable"
EV_METRICS_UNAVAILABLE = "MetricsUnavailable"


@dataclass(frozen=True)
class CanaryPolicy:
    """Reference constants (mlflow_operator.py:175-179,186-187,290-294) as defaults."""

    initial_traffic: int = 10
    step: int = 10
    interval_s: float = 60.0
    max_attempts: int = 10
    attempt_delay_s: float = 10.0
    rollback: bool = True           # reference: no rollback (":345"); README promises one
    thresholds: dict = field(default_factory=lambda: {
        "latency_95th": 0.05, "error_rate": 0.02, "latency_avg": 0.05})
    # absolute error-rate floor: with a 0 baseline the reference's relative test
    # demands exactly 0 errors; 0.0 reproduces the reference
    error_rate_floor: float = 0.0
    latency_floor_s: float = 0.0    # latencies below this always pass (0 = reference)
    window_s: int = 60              # PromQL range (mlflow_operator.py:363)
    ready_timeout_s: float = 1800.0  # wait for the new predictor's readiness before gating
    max_restarts: int = 3            # a canary predictor restarted this often is rolled back
    # GPU-side guards {metric: max new/old ratio} over prometheus.gpu_guard_queries;
    # skipped for predictors that do not export the series (reference runtimes)
    gpu_guards: dict = field(default_factory=lambda: {
        "tpot_avg": 1.10, "gpu_memory_used": 1.30, "gpu_power": 1.25,
        # kernel-time shares from the pods' in-process profiler (runtime.gpu_metrics)
        "attention_share": 1.5})

    @classmethod
    def from_spec(cls, spec: dict) -> "CanaryPolicy":
        c = (spec or {}).get("canary") or {}
        base = cls()
        th = dict(base.thresholds)
        th.update(c.get("thresholds") or {})
        return cls(initial_traffic=int(c.get("initialTraffic", base.initial_traffic)),
                   step=int(c.get("step", base.step)),
                   interval_s=float(c.get("intervalSeconds", base.interval_s)),
                   max_attempts=int(c.get("maxAttempts", base.max_attempts)),
                   attempt_delay_s=float(c.get("attemptDelaySeconds", base.attempt_delay_s)),
                   rollback=bool(c.get("rollback", base.rollback)),
                   thresholds=th,
                   error_rate_floor=float(c.get("errorRateFloor", base.error_rate_floor)),
                   latency_floor_s=float(c.get("latencyFloorSeconds", base.latency_floor_s)),
                   window_s=int(c.get("windowSeconds", base.window_s)),
                   ready_timeout_s=float(c.get("readyTimeoutSeconds", base.ready_timeout_s)),
                   max_restarts=int(c.get("maxRestarts", base.max_restarts)),
                   gpu_guards=dict(base.gpu_guards if c.get("gpuGuards") is None else c["gpuGuards"]))


@dataclass(frozen=True)
class ModelSpec:
    model_name: str
    model_alias: str
    monitoring_interval: float = 60.0
    minio_secret: str | None = None
    runtime: str | None = None
    architecture: str | None = None
    tensor_parallel: int | None = None
    expert_parallel: int | None = None
    replicas: int = 1
    max_model_len: int | None = None
    max_num_seqs: int | None = None
    kv_target_fraction: float | None = None
    canary: CanaryPolicy = field(default_factory=CanaryPolicy)

    @classmethod
    def from_spec(cls, spec: dict) -> "ModelSpec":
        spec = spec or {}
        return cls(model_name=spec.get("modelName"), model_alias=spec.get("modelAlias"),
                   monitoring_interval=float(spec.get("monitoringInterval", 60)),
                   minio_secret=spec.get("minioSecret"), runtime=spec.get("runtime"),
                   architecture=spec.get("architecture"),
                   tensor_parallel=spec.get("tensorParallel"),
                   expert_parallel=spec.get("expertParallel"),
                   replicas=int(spec.get("replicas", 1)),
                   max_model_len=spec.get("maxModelLen"), max_num_seqs=spec.get("maxNumSeqs"),
                   kv_target_fraction=spec.get("kvTargetFraction"),
                   canary=CanaryPolicy.from_spec(spec))

    def validate(self) -> list[str]:
        errs = []
        if not self.model_name:
            errs.append("spec.modelName is required")
        if not self.model_alias:
            errs.append("spec.modelAlias is required")
        if self.monitoring_interval <= 0:
            errs.append("spec.monitoringInterval must be > 0")
        return errs


@dataclass(frozen=True)
class OperatorSettings:
    """Operator-wide settings; defaults are the reference's hard-coded values."""

    prometheus_url: str = "http://seldon-monitoring-prometheus.seldon-monitoring.svc.cluster.local:9090"
    artifact_base: str = "s3://mlflow"
    runtime_image: str = "mlopamd/runtime-rocm:0.1.0"
    gpu_resource: str = "amd.com/gpu"
    hbm_per_gpu_gb: float = 288.0
    gpus_per_node: int = 8

    @classmethod
    def from_env(cls) -> "OperatorSettings":
        e = os.environ
        d = cls()
        return cls(prometheus_url=e.get("MLOP_PROMETHEUS_URL", d.prometheus_url),
                   artifact_base=e.get("MLOP_ARTIFACT_BASE", d.artifact_base),
                   runtime_image=e.get("MLOP_RUNTIME_IMAGE", d.runtime_image),
                   gpu_resource=e.get("MLOP_GPU_RESOURCE", d.gpu_resource),
                   hbm_per_gpu_gb=float(e.get("MLOP_HBM_PER_GPU_GB", d.hbm_per_gpu_gb)),
                   gpus_per_node=int(e.get("MLOP_GPUS_PER_NODE", d.gpus_per_node)))


def load_manifest(name: str) -> list[dict]:
    with open(MANIFESTS / name) as f:
        return [d for d in yaml.safe_load_all(f) if d]


def crd_schema() -> dict:
    crd = load_manifest("crd.yaml")[0]
    return crd["spec"]["versions"][0]["schema"]["openAPIV3Schema"]


def extract_relative_path(source_uri: str) -> str:
    """C2 (mlflow_operator.py:18-24): drop the ``mlflow-artifacts:/`` scheme and leading '/'."""
    prefix = "mlflow-artifacts:/"
    rel = source_uri[len(prefix):] if source_uri.startswith(prefix) else source_uri
    return rel.lstrip("/")


def artifact_uri(source: str, base: str = "s3://mlflow") -> str:
    """Reference URI rewrite (mlflow_operator.py:125-127); file:// sources kept for local runs."""
    if source.startswith("file://") or source.startswith("mlop://"):
        return source
    return f"{base.rstrip('/')}/{extract_relative_path(source)}"


# ---------------------------------------------- structural schema checks --
# What the kube-apiserver does with a CR body before storing it (structural
# OpenAPI v3 subset used by crd.yaml): reject type / bound / enum / required
# violations with 422 Invalid, prune fields the schema does not declare unless
# ``x-kubernetes-preserve-unknown-fields`` or ``additionalProperties`` allow them.
# The reference relies on the real apiserver for this (crd.yaml:11-37 there);
# the in-memory fake (kube.FakeKube) and its REST front-end apply it here.

_ROOT_FIELDS = ("apiVersion", "kind", "metadata")


def _type_ok(v, t: str) -> bool:
    if t == "object":
        return isinstance(v, dict)
    if t == "array":
        return isinstance(v, list)
    if t == "string":
        return isinstance(v, str)
    if t == "boolean":
        return isinstance(v, bool)
    if t == "integer":
        return isinstance(v, int) and not isinstance(v, bool)
    if t == "number":
        return isinstance(v, (int, float)) and not isinstance(v, bool)
    return True


def schema_errors(value, schema: dict, path: str = "") -> list[str]:
    """Field errors of ``value`` against a structural schema, kubectl-style
    (``spec.tensorParallel: Invalid value: 9: must be <= 8``)."""
    errs: list[str] = []
    where = path or "<root>"
    if value is None:
        if not schema.get("nullable", False) and path:
            errs.append(f"{where}: Invalid value: null: must not be null")
        return errs
    t = schema.get("type")
    if t and not _type_ok(value, t):
        return [f"{where}: Invalid value: {value!r}: must be of type {t}"]
    if "enum" in schema and value not in schema["enum"]:
        errs.append(f"{where}: Unsupported value: {value!r}: supported values: {schema['enum']}")
    if isinstance(value, (int, float)) and not isinstance(value, bool):
        if "minimum" in schema and value < schema["minimum"]:
            errs.append(f"{where}: Invalid value: {value}: must be >= {schema['minimum']}")
        if "maximum" in schema and value > schema["maximum"]:
            errs.append(f"{where}: Invalid value: {value}: must be <= {schema['maximum']}")
    if isinstance(value, dict):
        props = schema.get("properties", {})
        for req in schema.get("required", []):
            if req not in value:
                errs.append(f"{path + '.' if path else ''}{req}: Required value")
        extra = schema.get("additionalProperties")
        for k, v in value.items():
            sub = f"{path}.{k}" if path else k
            if k in props:
                errs += schema_errors(v, props[k], sub)
            elif isinstance(extra, dict):
                errs += schema_errors(v, extra, sub)
    if isinstance(value, list) and isinstance(schema.get("items"), dict):
        for i, v in enumerate(value):
            errs += schema_errors(v, schema["items"], f"{path}[{i}]")
    return errs


def prune(value, schema: dict, root: bool = True):
    """Drop undeclared fields (apiserver pruning); returns a new value."""
    if isinstance(value, dict):
        if schema.get("x-kubernetes-preserve-unknown-fields"):
            return dict(value)
        props = schema.get("properties", {})
        extra = schema.get("additionalProperties")
        out = {}
        for k, v in value.items():
            if root and k in _ROOT_FIELDS:
                out[k] = v
            elif k in props:
                out[k] = prune(v, props[k], root=False)
            elif isinstance(extra, dict):
                out[k] = prune(v, extra, root=False)
            elif extra is True:
                out[k] = v
        return out
    if isinstance(value, list) and isinstance(schema.get("items"), dict):
        return [prune(v, schema["items"], root=False) for v in value]
    return value


def admit(obj: dict, schema: dict | None = None) -> tuple[dict, list[str]]:
    """(pruned object, field errors) for an MlflowModel body, as the apiserver
    would store or reject it."""
    schema = schema or crd_schema()
    body = {k: v for k, v in obj.items() if k not in _ROOT_FIELDS}
    errs = schema_errors(body, schema)
    return prune(obj, schema), errs
