"""SeldonDeployment emission (reference C6/C6a/C7, mlflow_operator.py:156-286).

Wire contract kept from the reference: SD named after the CR, same namespace,
controller ownerReference (K8s GC cascades on CR delete), predictors named
``v{version}`` with graph ``classifier-{version}``, ``modelUri``,
``envSecretRefName``, ``replicas``, ``traffic``, ``protocol: kfserving``.

Predictor runtimes:
  * ``MLFLOW_SERVER`` — the reference's stock prepackaged server, emitted
    byte-compatible for users who ask for it explicitly;
  * ``mlop-llm`` — OUR PyTorch-ROCm LLM runtime (this package's
    ``mlopamd.runtime.server``): a componentSpec container requesting
    ``amd.com/gpu`` = TP degree, HBM-aware placement annotations, V2 readiness
    probe, the Seldon executor metric labels as env;
  * ``mlop-sklearn`` — the same server hosting CPU sklearn / pyfunc models
    (BASELINE config 1), replacing Seldon's MLServer.
"""
from __future__ import annotations

import copy

from .crd import API_VERSION, KIND, SELDON_GROUP, SELDON_KIND, SELDON_VERSION

RUNTIME_STOCK = "MLFLOW_SERVER"
RUNTIME_LLM = "mlop-llm"
RUNTIME_SKLEARN = "mlop-sklearn"
RUNTIMES = (RUNTIME_STOCK, RUNTIME_LLM, RUNTIME_SKLEARN)
ANN_PREFIX = "mlop.amd.com/"  # predictor annotations: runtime + the HBM-aware placement
POD_LABEL = "seldon-deployment-id"  # Seldon v1 labels every predictor pod with its SD's name


def predictor_name(version) -> str:
    return f"v{version}"


def graph_name(version) -> str:
    return f"classifier-{version}"


def owner_reference(body: dict) -> dict:
    md = body["metadata"]
    return {"apiVersion": body.get("apiVersion", API_VERSION), "kind": body.get("kind", KIND),
            "name": md["name"], "uid": md["uid"], "controller": True, "blockOwnerDeletion": True}


def build_predictor(version, model_uri: str, secret: str | None, traffic: int, runtime: str = RUNTIME_STOCK,
                    replicas: int = 1, placement: dict | None = None, image: str = "mlopamd/runtime-rocm:0.1.0",
                    gpu_resource: str = "amd.com/gpu", model_name: str | None = None,
                    deployment: str = "", namespace: str = "", architecture: str | None = None,
                    engine_args: dict | None = None) -> dict:
    graph = {"name": graph_name(version), "modelUri": model_uri, "envSecretRefName": secret, "children": []}
    pred = {"graph": graph, "name": predictor_name(version), "replicas": int(replicas), "traffic": int(traffic)}
    if runtime == RUNTIME_STOCK:
        graph["implementation"] = "MLFLOW_SERVER"
        return pred
    graph["type"] = "MODEL"
    graph["endpoint"] = {"type": "REST", "httpPort": 9000}
    tp = int((placement or {}).get("tensorParallel", 1))
    ep = int((placement or {}).get("expertParallel", 1))
    gpus = int((placement or {}).get("gpus", tp if runtime == RUNTIME_LLM else 0))
    # EP > 1 with TP = 1: data-parallel attention + expert-parallel MoE, one engine per GPU
    # behind one endpoint (runtime/ep_serving.py); EP = TP: experts sharded by the TP ranks
    par = ["--ep", str(ep)] if (tp == 1 and ep > 1) else ["--tp", str(tp)]
    env = [
        {"name": "MLOP_RUNTIME", "value": runtime},
        {"name": "MLOP_MODEL_URI", "value": model_uri},
        {"name": "MLOP_MODEL_NAME", "value": model_name or graph_name(version)},
        {"name": "MLOP_MODEL_VERSION", "value": str(version)},
        # the executor metric labels the reference's PromQL filters on
        {"name": "SELDON_DEPLOYMENT_ID", "value": deployment},
        {"name": "PREDICTOR_ID", "value": predictor_name(version)},
        {"name": "SELDON_NAMESPACE", "value": namespace},
        {"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"},
    ]
    if architecture:
        env.append({"name": "MLOP_ARCHITECTURE", "value": architecture})
    for k, v in (engine_args or {}).items():
        env.append({"name": f"MLOP_ENGINE_{k.upper()}", "value": str(v)})
    container = {
        "name": graph_name(version),
        "image": image,
        "command": ["python", "-m", "mlopamd.runtime.server"],
        "args": ["--port", "9000", *par],
        "env": env,
        "ports": [{"name": "http", "containerPort": 9000}],
        "readinessProbe": {"httpGet": {"path": "/v2/health/ready", "port": 9000},
                           "periodSeconds": 2, "failureThreshold": 1800},
        "livenessProbe": {"httpGet": {"path": "/v2/health/live", "port": 9000}, "periodSeconds": 10},
    }
    if gpus:
        container["resources"] = {"limits": {gpu_resource: str(gpus)}, "requests": {gpu_resource: str(gpus)}}
        container["volumeMounts"] = [{"name": "dshm", "mountPath": "/dev/shm"}]
    spec = {"containers": [container]}
    if gpus:
        spec["volumes"] = [{"name": "dshm", "emptyDir": {"medium": "Memory"}}]
    pred["componentSpecs"] = [{"spec": spec}]
    ann = {f"{ANN_PREFIX}runtime": runtime}
    for k, v in (placement or {}).items():
        ann[f"{ANN_PREFIX}{k}"] = str(v)
    pred["annotations"] = ann
    return pred


def build_seldon_deployment(name: str, namespace: str, owner_body: dict, predictors: list) -> dict:
    return {
        "apiVersion": f"{SELDON_GROUP}/{SELDON_VERSION}",
        "kind": SELDON_KIND,
        "metadata": {"name": name, "namespace": namespace, "ownerReferences": [owner_reference(owner_body)],
                     "labels": {"app.kubernetes.io/managed-by": "mlflow-operator"}},
        "spec": {"name": name, "protocol": "kfserving", "predictors": predictors},
    }


def spec_equal(a: dict, b: dict) -> bool:
    return (a or {}).get("spec") == (b or {}).get("spec")


def predictor_ready(sd: dict | None, predictor: str) -> bool:
    """True when the Seldon controller reports the predictor's deployment available."""
    if not sd:
        return False
    st = sd.get("status") or {}
    ds = st.get("deploymentStatus") or {}
    hits = [v for k, v in ds.items() if f"-{predictor}-" in k or k.endswith(f"-{predictor}")]
    if hits:
        return all(int(h.get("availableReplicas", 0)) >= max(1, int(h.get("replicas", 1))) for h in hits)
    names = [p["name"] for p in (sd.get("spec") or {}).get("predictors", [])]
    return st.get("state") == "Available" and names == [predictor]


def predictor_health(sd: dict | None, predictor: str) -> tuple[int, bool, str]:
    """(restarts, failed, reason) the Seldon controller reports for a predictor's
    deployments (pods that died and were restarted, or that could not start, e.g. a
    GPU out-of-memory at weight load)."""
    ds = ((sd or {}).get("status") or {}).get("deploymentStatus") or {}
    restarts, failed, reason = 0, False, ""
    for k, v in ds.items():
        if f"-{predictor}-" in k or k.endswith(f"-{predictor}"):
            restarts = max(restarts, int(v.get("restarts", 0)))
            failed = failed or bool(v.get("failed", False))
            reason = v.get("reason") or reason
    return restarts, failed, reason


def gpus_of(pred: dict, resource: str = "amd.com/gpu") -> int:
    """GPUs one replica of a predictor requests (container limits win over requests, as the
    scheduler reads them); 0 for the stock MLFLOW_SERVER predictor."""
    n = 0
    for cs in pred.get("componentSpecs") or []:
        for c in cs.get("spec", {}).get("containers", []):
            res = c.get("resources") or {}
            v = (res.get("limits") or {}).get(resource, (res.get("requests") or {}).get(resource, 0))
            n += int(v or 0)
    return n


def traffic_of(sd: dict | None) -> dict:
    return {p["name"]: p.get("traffic", 0) for p in ((sd or {}).get("spec") or {}).get("predictors", [])}


def with_traffic(sd: dict, weights: dict) -> dict:
    out = copy.deepcopy(sd)
    for p in out["spec"]["predictors"]:
        if p["name"] in weights:
            p["traffic"] = int(weights[p["name"]])
    return out
