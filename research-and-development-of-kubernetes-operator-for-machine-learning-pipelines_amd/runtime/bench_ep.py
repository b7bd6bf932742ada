"""The benchmark's expert-parallel phase: Mixtral-8x7B EP = world over the same GPUs (config 5).

After the Llama-3 DP replicas and the TP = N phase (runtime/bench_tp.py), ``bench.py --gpus N``
serves a short EP = N phase of Mixtral-8x7B in child processes, reported as the JSON line's
``ep`` block, so the one run on an N-GPU node also carries the expert exchange across devices
(CL4 over IPC peer memory, ops/csrc/ep_exchange.hip; RCCL all-to-all without it):

  1. every rank builds its EP shard: the dense weights (embedding, attention, router, norms)
     are drawn from the same seeded stream on every rank, and each expert's weights from a
     generator seeded by its GLOBAL expert id (``_init_experts``), so the N shards are exactly
     one model whose experts are all different (a dispatch to the wrong rank changes tokens);
  2. greedy check (``_check``) at the model's full width and CHECK_LAYERS depth: 8 fixed prompts
     x ``CHECK_TOKENS`` tokens through the EP group's engines (rank 0 serves them, the others
     join with padding-only forwards: DP attention, every MoE layer an exchange over the whole
     group); rank 0 then holds the same model whole (EP = 1) and checks the tokens against the
     dense fp32 oracle (models/reference.py; top 16 and within 1 logit std, MOE_MAX_RANK,
     bench_tp._dense_agreement) and against an EP = 1 engine;
  3. a closed-loop serve of the FULL-depth shard, ``--ep-batch`` requests PER RANK,
     ``--tp-warmup`` + ``--tp-steps`` steps timed between syncs and world barriers ->
     ``tokens_per_sec`` (all ranks).
"""
from __future__ import annotations

import gc
import os
import sys
import threading
import time

import torch

from .bench_tp import PROMPTS, _clamp_prompts, _dense_agreement

CHECK_TOKENS = 2
CHECK_LAYERS = 2
# the oracle bound for MoE tokens: top 16 of 32k ids and within 1 logit std. Wider than the dense
# models' (top 5, 0.25 std): a router top-2 flip on one prompt token (bf16 vs fp32 routing logits)
# moves the last logits more than bf16 summation noise does. Measured on Mixtral-8x7B at 2 layers:
# the worst bf16 token at rank 5 / 0.64 std, identical for the EP = 1 engine (same tokens 16/16).
# A wrong dispatch / combine lands at a random rank: inside the bound with p = 16 / 32k per token.
MOE_MAX_RANK, MOE_MAX_GAP = 16, 1.0


@torch.no_grad()
def _init_experts(model, seed: int) -> None:
    """Expert e of layer l <- N(0, 0.02) from a generator seeded by (seed, l, e): the same values
    whichever rank (or the full model) holds expert e."""
    for li, L in enumerate(model.layers):
        for j in range(model.n_local_experts):
            e = model.expert_start + j
            g = torch.Generator(device=model.device).manual_seed(seed * 7919 + li * 1024 + e)
            for name in ("w13", "w2"):
                t = L[name][j]
                t.copy_(torch.empty(t.shape, device=model.device, dtype=torch.float32).normal_(0.0, 0.02, generator=g)
                        .to(t.dtype))


@torch.no_grad()
def _copy_dense(dst, src) -> None:
    """dst (EP = 1) <- src's dense weights (EP shard of the same config): everything but experts."""
    dst.embed.copy_(src.embed)
    for Ld, Ls in zip(dst.layers, src.layers):
        for k in Ld:
            if k not in ("w13", "w2"):
                Ld[k].copy_(Ls[k])
    dst.final_norm.copy_(src.final_norm)
    if dst.lm_head is not dst.embed:
        dst.lm_head.copy_(src.lm_head)


def _check(a, rank: int, dev, dtype, cfg, ps, seed: int) -> dict:
    """Greedy check of the EP group on ``cfg`` (the bench model's width at CHECK_LAYERS depth).

    Every rank builds its shard and an engine and steps ``generate`` together (rank 0 with the
    prompts, the others padding-only forwards that still join every exchange). Rank 0 then holds
    the same model whole (EP = 1) and returns (others: {}):
      * the dense fp32 oracle's verdict on the EP tokens (bench_tp._dense_agreement);
      * ``tokens_equal_ep1_engine``: EP tokens equal to an EP = 1 engine's on the whole model
        (the same kernels without the exchange).

    Why not full depth: a random-init Mixtral's greedy tokens are chaotic in depth. Rounding only
    the MoE input to bf16 in the fp32 oracle flips 10 of 8,320 router top-2 selections over 32
    layers and moves the oracle's own argmax to rank 133-210 (profiles/r06_ep_phase.md,
    scripts/ep_chaos_probe.py); any bf16 engine, EP or not, then lands at rank ~2,000. At 2
    layers no selection flips, the engine agrees 15/16 exactly, and a wrong dispatch or
    combine gives a token at a random rank of 32k."""
    from ..models import build_model
    from .engine import Engine, EngineConfig
    from .sampler import SamplingParams

    shard = build_model(cfg, device=dev, dtype=dtype, pstate=ps, seed=seed)
    _init_experts(shard, seed)
    prompts = _clamp_prompts(PROMPTS, cfg.vocab_size)
    ec = dict(max_num_seqs=len(prompts), max_num_batched_tokens=a.max_batched_tokens, max_model_len=a.max_model_len,
              num_kv_blocks=len(prompts) * 8 + 16, use_graphs=not a.no_graphs, graph_buckets=(len(prompts),),
              async_scheduling=False)
    eng = Engine(shard, EngineConfig(**ec))
    exchange = "ipc" if getattr(ps.ep, "ex", None) is not None else "all_to_all"
    toks = eng.generate(prompts if rank == 0 else [], SamplingParams(max_tokens=CHECK_TOKENS, ignore_eos=True))
    eng.shutdown()
    del eng
    if rank != 0:
        return {}
    out = {"exchange": exchange, "check_layers": cfg.num_layers}
    full = build_model(cfg, device=dev, dtype=dtype, seed=seed)
    _copy_dense(full, shard)
    _init_experts(full, seed)
    out.update(_dense_agreement(full, prompts, toks, max_rank=MOE_MAX_RANK, max_gap=MOE_MAX_GAP))
    e1 = Engine(full, EngineConfig(**ec))
    ref = e1.generate(prompts, SamplingParams(max_tokens=CHECK_TOKENS, ignore_eos=True))
    e1.shutdown()
    out["tokens_equal_ep1_engine"] = sum(int(x == y) for p_, q_ in zip(toks, ref) for x, y in zip(p_, q_))
    return out


def ep_phase(a, rank: int, world: int, dev, serve, on_fail) -> dict | None:
    """Run the EP = world phase on every rank; rank 0 returns the ``ep`` block (others None)."""
    import torch.distributed as dist

    from ..models import build_model
    from ..models.config import get_config
    from ..parallel.comm import make_parallel_state
    from .engine import Engine, EngineConfig
    from .kv_cache import blocks_needed

    t_phase = time.perf_counter()
    done = threading.Event()

    def watchdog():
        if done.wait(a.tp_timeout):
            return
        msg = f"EP phase exceeded --tp-timeout {a.tp_timeout:.0f} s"
        print(f"[bench rank {rank}] {msg}: exiting", file=sys.stderr, flush=True)
        on_fail(msg)
        os._exit(3)

    threading.Thread(target=watchdog, daemon=True, name="ep-phase-watchdog").start()
    out: dict = {"ep": world, "world": world, "model": a.ep_model}
    try:
        gc.collect()
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
            torch.cuda.empty_cache()
        dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
        cfg = get_config(a.ep_model)
        seed = a.seed + 91
        ps = make_parallel_state(tp_size=1, ep_size=world)
        out["backend"] = dist.get_backend() if dist.is_initialized() else None
        # 1. greedy check at CHECK_LAYERS depth (full width, every MoE layer an exchange)
        t0 = time.perf_counter()
        out.update(_check(a, rank, dev, dtype, get_config(a.ep_model, num_layers=min(cfg.num_layers, CHECK_LAYERS)),
                          ps, seed))
        out["check_s"] = round(time.perf_counter() - t0, 2)
        gc.collect()
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
            torch.cuda.empty_cache()
        # 2. the timed serve on the full-depth shard
        t0 = time.perf_counter()
        shard = build_model(cfg, device=dev, dtype=dtype, pstate=ps, seed=seed)
        _init_experts(shard, seed)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        out["build_s"] = round(time.perf_counter() - t0, 2)
        out["weight_gb_per_gpu"] = round(shard.weight_bytes() / 1e9, 3)
        B = a.ep_batch
        nb = B * blocks_needed(min(a.max_model_len, a.prompt_len + a.output_len + 16)) + 64
        ec = EngineConfig(max_num_seqs=B, max_num_batched_tokens=a.max_batched_tokens,
                          max_model_len=a.max_model_len, num_kv_blocks=nb, use_graphs=not a.no_graphs,
                          prefill_min_batch=a.prefill_min_batch, max_decode_gap=a.max_decode_gap,
                          mixed_prefill=not a.no_mixed, mixed_min_chunk=a.mixed_min_chunk,
                          enable_prefix_caching=not a.no_prefix_cache)
        t0 = time.perf_counter()
        eng = Engine(shard, ec)
        out["engine_s"] = round(time.perf_counter() - t0, 2)
        out["exchange"] = "ipc" if getattr(ps.ep, "ex", None) is not None else "all_to_all"
        gen, elapsed, stats, ramp = serve(eng, a, a.ep_batch, a.tp_steps, a.tp_warmup, rank, ep_group=ps.ep_cpu)
        t_all = torch.tensor([float(gen), elapsed], dtype=torch.float64)
        if dist.is_initialized():
            parts = [torch.zeros_like(t_all) for _ in range(world)]
            dist.all_gather(parts, t_all, group=ps.ep_cpu)
        else:
            parts = [t_all]
        if rank != 0:
            out = None
        else:
            tot = sum(float(p[0]) for p in parts)
            t_max = max(float(p[1]) for p in parts)
            out.update({"batch_per_rank": a.ep_batch, "steps": a.tp_steps, "warmup": a.tp_warmup, "ramp_steps": ramp,
                        "tokens_per_sec": round(tot / max(t_max, 1e-9), 2),
                        "ms_per_step": round(1e3 * t_max / max(1, a.tp_steps), 3),
                        "graph_steps": int(stats.get("graph_steps", 0))})
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        if dist.is_initialized():
            dist.barrier()
        if out is not None:
            out["wall_s"] = round(time.perf_counter() - t_phase, 2)
        return out
    except Exception as e:  # noqa: BLE001 - reported in the line; the DP value stands
        import traceback

        traceback.print_exc()
        on_fail(f"{type(e).__name__}: {e}"[:500])
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(4)
    finally:
        done.set()
