"""Tensor-parallel predictor process group (config 4: Llama-3-70B TP=8).

One process per GPU.  The predictor container's command is plain
``python -m mlopamd.runtime.server --tp N`` (controller/seldon.py): started without
``WORLD_SIZE`` it becomes the launcher of N rank processes (``server.launch_ranks``);
``torchrun --nproc-per-node N -m mlopamd.runtime.server ...`` works the same way.  Every
rank builds its shard of the model (Megatron column/row/vocab-parallel, RCCL all-reduce
over xGMI) and an identical engine; rank 0 alone serves HTTP and schedules, broadcasting
each step's metadata (``engine.StepSync``); ranks > 0 sit in ``worker_loop``.
"""
from __future__ import annotations

import os

import torch


def build_tp_engine(architecture: str, tp: int, device=None, seed: int = 0, engine_kwargs: dict | None = None,
                    full_model=None, model_uri: str | None = None, ep: int | None = None):
    """``ep``: expert-parallel degree of a MoE model (default = tp: experts sharded over the
    TP ranks, partial outputs summed by the TP all-reduce)."""
    from ..models import build_model
    from ..parallel.comm import init_distributed, make_parallel_state
    from .engine import Engine, EngineConfig

    from .rank_launcher import share_gpu_requested

    # one-GPU rehearsal of a multi-rank pod (rank_launcher.py): every rank on device 0, gloo
    # (RCCL refuses two ranks on one device), the IPC kernels forced by the launcher's env
    share = share_gpu_requested([])
    if device is None:
        local = 0 if share else int(os.environ.get("LOCAL_RANK", 0))
        device = torch.device("cuda", local) if torch.cuda.is_available() else "cpu"
    device = torch.device(device)
    if device.type == "cuda":
        torch.cuda.set_device(device)
    init_distributed(backend="gloo" if (device.type == "cpu" or share) else None)
    ps = make_parallel_state(tp_size=tp, ep_size=ep or tp)
    from ..models.loader import load_pretrained, resolve_model_dir

    dtype = torch.bfloat16 if device.type == "cuda" else torch.float32
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
    """Entry from ``runtime.server.main`` when WORLD_SIZE > 1 (one call per rank)."""
    from aiohttp import web

    from .backends import LLMBackend
    from .server import engine_kwargs_from_env, make_app

    tp = int(os.environ.get("WORLD_SIZE", args.tp))
    rank = int(os.environ.get("RANK", 0))
    if rank == 0 and os.environ.get("MLOP_INJECT_START_ERROR"):  # fault injection, as for TP=1
        raise RuntimeError(os.environ["MLOP_INJECT_START_ERROR"])
    device = None
    if args.device == "cpu" or not torch.cuda.is_available():
        device = "cpu"
    eng, ps = build_tp_engine(args.architecture or "llama3-70b", tp, device=device,
                              engine_kwargs=engine_kwargs_from_env(), model_uri=args.model_uri,
                              seed=int(os.environ.get("MLOP_SEED", 0)))
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
