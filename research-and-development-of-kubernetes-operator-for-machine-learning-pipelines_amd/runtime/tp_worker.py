"""Tensor-parallel predictor process group (config 4: Llama-3-70B TP=8).

Launched as one process per GPU (``torchrun --nproc-per-node TP -m
mlopamd.runtime.server ...``).  Every rank builds its shard of the model
(Megatron column/row/vocab-parallel, RCCL all-reduce over xGMI) and an
identical engine; rank 0 alone serves HTTP and schedules, broadcasting each
step's metadata (``engine.StepSync``); ranks > 0 sit in ``worker_loop``.
"""
from __future__ import annotations

import os

import torch


def build_tp_engine(architecture: str, tp: int, device=None, seed: int = 0, engine_kwargs: dict | None = None,
                    full_model=None, model_uri: str | None = None):
    from ..models import build_model
    from ..parallel.comm import init_distributed, make_parallel_state
    from .engine import Engine, EngineConfig

    init_distributed()
    ps = make_parallel_state(tp_size=tp, ep_size=tp)
    if device is None:
        device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0))) if torch.cuda.is_available() else "cpu"
    from ..models.loader import load_pretrained, resolve_model_dir

    dtype = torch.bfloat16 if torch.device(device).type == "cuda" else torch.float32
    ckpt = resolve_model_dir(model_uri)
    if ckpt is not None:  # every rank reads only its own shard of the checkpoint
        model = load_pretrained(ckpt, device=device, dtype=dtype, pstate=ps)
    else:
        model = build_model(architecture, device=device, pstate=ps, seed=seed, dtype=dtype)
    if full_model is not None:
        model.load_shard_from(full_model)
    eng = Engine(model, EngineConfig(**(engine_kwargs or {})))
    eng.checkpoint_dir = ckpt
    return eng, ps


def serve_tp(args, metrics):
    """Entry from ``runtime.server.main`` when WORLD_SIZE > 1."""
    from aiohttp import web

    from .backends import LLMBackend
    from .server import engine_kwargs_from_env, make_app

    tp = int(os.environ.get("WORLD_SIZE", args.tp))
    eng, ps = build_tp_engine(args.architecture or "llama3-70b", tp, engine_kwargs=engine_kwargs_from_env(),
                              model_uri=args.model_uri)
    if ps.tp_rank != 0:
        eng.worker_loop()
        return
    from .backends import load_tokenizer

    backend = LLMBackend(eng, metrics, tokenizer=load_tokenizer(eng.checkpoint_dir), name=args.name).start()
    try:
        web.run_app(make_app(backend, metrics, version=args.version), host=args.host, port=args.port, print=None)
    finally:
        backend.stop()
        eng.shutdown()
