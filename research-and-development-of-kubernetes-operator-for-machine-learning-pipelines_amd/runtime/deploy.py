"""Runtime construction: model + engine from a model name / predictor spec.

``build_engine`` is what a predictor process runs at start-up (random-init
weights on device, KV cache sized for 288 GB HBM, decode hipGraph capture).
``deploy_for_bench`` drives the same start-up through the control plane when
the operator is available (CR -> SeldonDeployment -> in-process predictor ->
ready), returning the CR->ready time the headline metric reports.
"""
from __future__ import annotations

import time

import torch

from ..models import build_model
from .engine import Engine, EngineConfig


def build_engine(model: str = "llama3-8b", device="cuda", seed: int = 0, tp_state=None,
                 dtype=torch.bfloat16, model_uri: str | None = None, **engine_kwargs) -> Engine:
    """Weights from the predictor's artifact when it is a local HF checkpoint
    (``models.loader.resolve_model_dir``), else random-init ``model`` (the benchmark)."""
    from ..models.loader import load_pretrained, resolve_model_dir

    t0 = time.perf_counter()
    ckpt = resolve_model_dir(model_uri)
    if ckpt is not None:
        m = load_pretrained(ckpt, device=device, dtype=dtype, pstate=tp_state)
    else:
        m = build_model(model, device=device, dtype=dtype, pstate=tp_state, seed=seed)
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)
    t1 = time.perf_counter()
    eng = Engine(m, EngineConfig(**engine_kwargs))
    eng.stats["model_build_ms"] = int(1e3 * (t1 - t0))
    eng.checkpoint_dir = ckpt  # None: random-init weights
    return eng


def deploy_for_bench(model: str, device, use_operator: bool = True, seed: int = 0,
                     engine_kwargs: dict | None = None):
    engine_kwargs = engine_kwargs or {}
    if use_operator:
        try:
            from ..controller.local import deploy_and_wait
        except ImportError:  # control plane not importable: direct start-up
            use_operator = False
    t0 = time.perf_counter()
    if use_operator:
        engine, info = deploy_and_wait(model=model, device=device, seed=seed, engine_kwargs=engine_kwargs)
        ready = time.perf_counter() - t0
        info["path"] = "operator"
        return engine, ready, info
    engine = build_engine(model, device=device, seed=seed, **engine_kwargs)
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize()
    ready = time.perf_counter() - t0
    return engine, ready, {"path": "direct", "weight_gb": round(engine.model.weight_bytes() / 1e9, 2),
                           "kv_blocks": engine.kv.num_blocks}
