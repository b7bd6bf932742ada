"""The benchmark's tensor-parallel phase: TP = world over the same ranks as the DP replicas.

``bench.py --gpus N`` measures N data-parallel Llama-3 replicas (the reference's predictor
``replicas``, /root/reference/mlflow_operator.py:204-205,219-220), whose only collective is
the result gather.  So that the one run on an N-GPU node also says something about configs 4
and 5 (TP over RCCL + xGMI), the same ranks then free their DP engines and serve a short
TP = N phase of the same model, reported as the JSON line's ``tp`` block:

  1. every rank random-initialises the FULL model (same seed: identical weights on every
     device, on-device RNG) and copies its Megatron shard out of it (``load_shard_from``);
  2. the TP group is built over the RCCL process group with the K15 IPC all-reduce, whose
     start-up self-check (parallel/custom_ar.py ``self_check``: exact rank-order sums of
     seeded inputs, one-shot / two-shot / add / broadcast / gather) must pass on EVERY rank,
     else the whole group falls back to the process-group collectives (``k15: "fallback"``);
  3. greedy check: 8 fixed prompts, 4 tokens each, through the TP engine (prefill eager,
     decode steps in hipGraphs with K15 inside); rank 0 then recomputes every step with the
     dense fp32 TP = 1 oracle (models/reference.py) on the full model and requires each token
     to sit in the oracle's top 5 within 0.25 logit stds of its argmax (``_dense_agreement``:
     bf16 noise flips near-tied argmaxes, a broken reduction lands at a random rank) ->
     ``first_token_match`` / ``tokens_match``; the same prompts through a TP = 1 engine on
     rank 0 give the bf16 noise floor beside it (``tp1_engine_vs_dense``);
  4. a closed-loop serve of ``--tp-batch`` requests, ``--tp-warmup`` + ``--tp-steps`` engine
     steps timed between device syncs + world barriers -> ``tokens_per_sec``.

bench.py runs the phase in child processes (``--phase-child tp``), one per rank with its own
process group, so a first-contact failure on real peers -- a hang, an abort, a GPU fault --
ends the children, never the DP ranks that hold the line's value.  A watchdog bounds the
phase inside the children (``--tp-timeout``) and the parents kill a child past it + 60 s.
"""
from __future__ import annotations

import gc
import os
import sys
import threading
import time

import torch

# 8 fixed prompts (BOS + a run of ids, 8-65 tokens; reduced modulo a smaller vocabulary)
PROMPTS = [[128000] + list(range(1000 + 37 * i, 1000 + 37 * i + n)) for i, n in
           enumerate((7, 12, 19, 26, 33, 40, 51, 64))]
CHECK_TOKENS = 4


def _dense_agreement(full, prompts, outs, max_rank: int = 5, max_gap: float = 0.25):
    """Teacher-forced along the engine's own tokens: for every generated token, its rank among the
    dense fp32 TP = 1 logits (0 = the argmax) and its logit gap to the argmax in logit stds.

    Random-init Llama-3 logits over 128k ids are near-Gaussian, so the top-2 gap is often ~0.1
    std and bf16 summation-order noise (TP, or just bf16 vs fp32) flips exact argmaxes; a wrong
    all-reduce instead produces unrelated logits, whose token lands at a uniformly random rank
    (top-5 by chance: 5 / 128k).  A token agrees when it is within the dense top ``max_rank``
    AND within ``max_gap`` stds of the argmax."""
    from ..models.reference import dense_logits

    first, agree, exact, worst_gap, worst_rank = [], 0, 0, 0.0, 0
    for p, o in zip(prompts, outs):
        toks = list(p)
        for j, t in enumerate(o):
            lg = dense_logits(full, toks)[-1]
            best = int(lg.argmax())
            gap = float(lg[best] - lg[t]) / max(float(lg.std()), 1e-12)
            rank = int((lg > lg[t]).sum())
            ok = rank < max_rank and gap < max_gap
            exact += int(t == best)
            agree += int(ok)
            worst_gap, worst_rank = max(worst_gap, gap), max(worst_rank, rank)
            if j == 0:
                first.append(ok)
            toks.append(t)
    n = sum(len(o) for o in outs)
    return {"first_token_match": bool(first) and all(first), "tokens_match": agree == n,
            "tokens_checked": n, "tokens_exact": exact, "worst_gap_in_std": round(worst_gap, 4),
            "worst_rank": worst_rank}


def _tp1_engine_tokens(full, prompts, a):
    """The same prompts through a TP = 1 engine on rank 0 (same HIP kernels, no collectives):
    the bf16 noise floor the TP tokens are read against."""
    from .engine import Engine, EngineConfig
    from .sampler import SamplingParams

    eng = Engine(full, EngineConfig(max_num_seqs=len(prompts), max_num_batched_tokens=a.max_batched_tokens,
                                    max_model_len=a.max_model_len, num_kv_blocks=len(prompts) * 8 + 16,
                                    use_graphs=not a.no_graphs, graph_buckets=(len(prompts),),
                                    async_scheduling=False))
    out = eng.generate(prompts, SamplingParams(max_tokens=CHECK_TOKENS, ignore_eos=True))
    eng.shutdown()
    return out


def _clamp_prompts(prompts, vocab):
    return [[t % vocab for t in p] for p in prompts]


def tp_phase(a, rank: int, world: int, dev, serve, on_fail) -> dict | None:
    """Run the TP = world phase on every rank; rank 0 returns the ``tp`` block (others None).
    ``serve``: bench.serve_closed_loop; ``on_fail(msg)``: called by the watchdog or on an
    exception, right before this process exits (bench.py runs the phase in child processes
    whose rank 0 writes the block, or that message, to a file its parent reads)."""
    import torch.distributed as dist

    from ..models import build_model
    from ..models.config import get_config
    from ..parallel.comm import make_parallel_state
    from .engine import Engine, EngineConfig
    from .kv_cache import blocks_needed
    from .sampler import SamplingParams

    t_phase = time.perf_counter()
    done = threading.Event()

    def watchdog():
        if done.wait(a.tp_timeout):
            return
        msg = f"TP phase exceeded --tp-timeout {a.tp_timeout:.0f} s (first-contact hang?)"
        print(f"[bench rank {rank}] {msg}: exiting", file=sys.stderr, flush=True)
        on_fail(msg)
        os._exit(3)

    threading.Thread(target=watchdog, daemon=True, name="tp-phase-watchdog").start()
    if os.environ.get("MLOP_INJECT_TP_PHASE_ABORT") == str(rank):  # fault injection: this rank dies
        os.abort()
    out: dict = {"tp": world, "world": world}
    try:
        gc.collect()
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
            torch.cuda.empty_cache()
        dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
        cfg = get_config(a.model)
        t0 = time.perf_counter()
        full = build_model(cfg, device=dev, dtype=dtype, seed=a.seed + 77)
        ps = make_parallel_state(tp_size=world)
        out["backend"] = dist.get_backend() if dist.is_initialized() else None
        out["k15"] = ps.tp.car_status
        chk = ps.tp.car_check or {}
        out["k15_check"] = {k: v for k, v in chk.items() if k in ("checks", "error_word", "exception")}
        shard = build_model(cfg, device=dev, dtype=dtype, pstate=ps, seed=a.seed + 77).load_shard_from(full)
        if rank != 0:  # rank 0 keeps the full model for the dense TP = 1 recompute
            del full
            full = None
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        out["build_s"] = round(time.perf_counter() - t0, 2)
        out["weight_gb_per_gpu"] = round(shard.weight_bytes() / 1e9, 3)
        B = max(len(PROMPTS), a.tp_batch)
        nb = B * blocks_needed(min(a.max_model_len, a.prompt_len + a.output_len + 16)) + 64
        ec = EngineConfig(max_num_seqs=B, max_num_batched_tokens=a.max_batched_tokens,
                          max_model_len=a.max_model_len, num_kv_blocks=nb, use_graphs=not a.no_graphs,
                          prefill_min_batch=a.prefill_min_batch, max_decode_gap=a.max_decode_gap,
                          mixed_prefill=not a.no_mixed, mixed_min_chunk=a.mixed_min_chunk,
                          enable_prefix_caching=not a.no_prefix_cache)
        t0 = time.perf_counter()
        eng = Engine(shard, ec)
        out["engine_s"] = round(time.perf_counter() - t0, 2)
        out["graph_capture_ms"] = eng.stats.get("graph_capture_ms", 0)
        if ps.tp_rank != 0:
            eng.worker_loop()  # the greedy check, then the serve: until the leader's STOP
            out = None
        else:
            prompts = _clamp_prompts(PROMPTS, cfg.vocab_size)
            toks = eng.generate(prompts, SamplingParams(max_tokens=CHECK_TOKENS, ignore_eos=True))
            gen, elapsed, stats, ramp = serve(eng, a, a.tp_batch, a.tp_steps, a.tp_warmup, rank)
            eng.shutdown()
            out.update({"batch": a.tp_batch, "steps": a.tp_steps, "warmup": a.tp_warmup, "ramp_steps": ramp,
                        "tokens_per_sec": round(gen / max(elapsed, 1e-9), 2),
                        "ms_per_step": round(1e3 * elapsed / max(1, a.tp_steps), 3),
                        "graph_steps": int(stats.get("graph_steps", 0)),
                        "decode_tokens": int(stats.get("decode_tokens", 0)),
                        "prefill_tokens": int(stats.get("prefill_tokens", 0))})
            t0 = time.perf_counter()
            out.update(_dense_agreement(full, prompts, toks))
            ref = _tp1_engine_tokens(full, prompts, a)
            out["tp1_engine_vs_dense"] = _dense_agreement(full, prompts, ref)
            out["first_tokens_equal_tp1_engine"] = sum(int(x[0] == y[0]) for x, y in zip(toks, ref))
            out["check_s"] = round(time.perf_counter() - t0, 2)
        err = ps.tp.car.error() if ps.tp.car is not None else 0
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        if dist.is_initialized():
            dist.barrier()
        if ps.tp.car is not None:
            ps.tp.car.close()
        if out is not None:
            out["k15_error_word"] = err
            out["wall_s"] = round(time.perf_counter() - t_phase, 2)
        return out
    except Exception as e:  # noqa: BLE001 - reported in the line; the DP value stands
        import traceback

        traceback.print_exc()
        msg = f"{type(e).__name__}: {e}"
        on_fail(msg[:500])
        # peers may be blocked in a collective with us: leave now, their watchdogs end them
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(4)
    finally:
        done.set()
