#!/usr/bin/env python3
"""Headline benchmark: served tokens/s on an auto-deployed Llama-3-8B (+ p50 CR->ready).

BASELINE.json metric: "served tokens/sec/MI355X on auto-deployed Llama-3-8B +
p50 CR-reconcile->ready".  Each rank (one process per GPU, launched by
torch.distributed.run for N > 1) is one data-parallel serving replica (the
reference's predictor ``replicas``; Llama-3-8B bf16 = 16 GB fits one 288 GB
MI355X, so replicas scale weakly with N):

  1. deploy: an ``MlflowModel`` CR is reconciled by the operator into a
     SeldonDeployment whose predictor is this runtime; the runtime
     random-initialises Llama-3-8B bf16 on the GPU, captures its decode
     hipGraphs and reports ready -> CR->ready seconds (p50 over ranks);
  2. serve: a closed-loop load of ``--batch`` concurrent requests
     (``--prompt-len`` random prompt tokens, ``--output-len`` generated tokens,
     the first cohort at staggered ages so the engine is in steady state),
     continuous batching with chunked prefill and graph-replayed decode;
  3. time exactly ``--steps`` engine steps after ``--warmup`` untimed ones,
     bracketed by barrier + device synchronize; value = generated tokens over
     all ranks / max rank time.

Synthetic data, random-init weights (no checkpoints / datasets offline).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs of this node to use; > 1 without a torch.distributed launcher (no WORLD_SIZE in "
                         "the env): this process becomes the launcher of N rank processes, one per GPU, "
                         "before it makes any HIP call")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=2048,
                    help="concurrent requests per GPU: 288 GB of HBM holds their ~100 GB of KV pages, and "
                         "~4k-row mixed steps keep the MFMA GEMMs near their large-M rate")
    ap.add_argument("--prompt-len", type=int, default=256)
    ap.add_argument("--output-len", type=int, default=256)
    ap.add_argument("--max-model-len", type=int, default=1024)
    # per-step token budget (decode rows + prompt chunks) and how many queued prompts start a
    # mixed step: 10240 / 8 measured +4.2 % over 8192 / 4 in one process-interleaved A/B
    # (scripts/run118-121.sh: 33.6k vs 32.2k tok/s; 12288 and prefill_min_batch 12 lose)
    ap.add_argument("--max-batched-tokens", type=int, default=10240)
    ap.add_argument("--prefill-min-batch", type=int, default=8)
    ap.add_argument("--max-decode-gap", type=int, default=24)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-async", action="store_true",
                    help="synchronous scheduling (default: step t+1 is launched before step t's tokens are read)")
    ap.add_argument("--no-mixed", action="store_true",
                    help="separate prefill steps instead of prompt chunks riding in the decode step")
    ap.add_argument("--mixed-min-chunk", type=int, default=64)
    ap.add_argument("--no-ramp", dest="ramp", action="store_false",
                    help="start warmup right after submitting the first cohort (prefill-heavy first steps)")
    ap.add_argument("--no-operator", action="store_true", help="skip the CR->SeldonDeployment deploy path")
    ap.add_argument("--temperature", type=float, default=0.0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--shared-prefix", type=int, default=0,
                    help="the first N prompt tokens are the same for every request (a system prompt): "
                         "exercises the prefix cache; 0 = fully random prompts (the headline)")
    ap.add_argument("--no-prefix-cache", action="store_true")
    ap.add_argument("--tune-in-timed", action="store_true",
                    help="keep timing first-seen GEMM shapes during the timed steps (default: frozen after warmup)")
    ap.add_argument("--save-gemm-table", default=None,
                    help="after the run, write the per-shape GEMM backend choices measured here to this JSON")
    ap.add_argument("--tp", type=int, default=1,
                    help="tensor-parallel degree per replica (config 4: --model llama3-70b --tp 8); "
                         "replicas = world / tp, each TP group's rank 0 schedules")
    ap.add_argument("--ep", type=int, default=1,
                    help="expert-parallel degree (config 5: --model mixtral-8x7b --ep N): N data-parallel "
                         "attention engines, each rank serving its own --batch requests, every MoE layer an "
                         "expert exchange over IPC peer memory (parallel/ep_ipc.py); replicas = world / ep")
    ap.add_argument("--share-gpu", action="store_true",
                    help="every rank on cuda:0 (gloo process group; RCCL cannot put two ranks on one GPU): "
                         "rehearses the multi-rank paths (EP exchange, TP K15 all-reduce) on a one-GPU box")
    ap.add_argument("--kv-gb", type=float, default=None,
                    help="KV-cache pool per rank in GB (default: sized from free HBM; set it with --share-gpu)")
    ap.add_argument("--http", action="store_true",
                    help="drive the load through the deployed stack instead: operator + ProcessLauncher "
                         "(a fresh predictor process: CR->ready includes its start-up) + V2 HTTP + Router "
                         "(runtime/http_bench.py); the value is the served rate over the predictor's own "
                         "engine steps")
    ap.add_argument("--http-check", type=int, default=-1,
                    help="also measure the served rate over HTTP at this config (a fresh predictor process "
                         "through operator + ProcessLauncher + V2 clients, runtime/http_bench.py) BEFORE the "
                         "engine-direct run, and report it as served_tokens_per_sec_http; its window is "
                         "max(--steps, 40) engine steps.  -1 (default): on for the 1-GPU operator bench, "
                         "off otherwise; 0 / 1 force it")
    ap.add_argument("--ab-ops", default="",
                    help="A/B runs: comma list of op=value set through torch.ops.mlop before the engine "
                         "is built, e.g. gemm_half_tile=0 (in-process switches, scripts/ab.sh)")
    ap.add_argument("--tp-phase", choices=("auto", "on", "off"), default="auto",
                    help="after the DP replicas (the line's value), run a short TP = world phase of the same "
                         "model on the same ranks: RCCL process group + the K15 IPC all-reduce across the "
                         "devices (xGMI), with K15's start-up self-check and a greedy-token check against a "
                         "dense TP = 1 recompute, reported as the 'tp' block.  auto: on when world > 1")
    ap.add_argument("--tp-batch", type=int, default=256, help="concurrent requests of the TP phase")
    ap.add_argument("--tp-steps", type=int, default=10, help="timed engine steps of the TP phase")
    ap.add_argument("--tp-warmup", type=int, default=3)
    ap.add_argument("--tp-timeout", type=float, default=240.0,
                    help="time limit of ONE phase (TP or EP; seconds): its child processes stop past it and the "
                         "line carries tp.error / ep.error, so a first-contact hang cannot eat the DP result")
    ap.add_argument("--phase-budget", type=float, default=240.0,
                    help="wall-time budget of the TP and EP phases together (seconds): a phase gets at most "
                         "what is left of it (a phase with < 30 s left is skipped and says so), so a hang in "
                         "the first phase cannot push the whole command past the driver's time limit")
    ap.add_argument("--ep-phase", choices=("auto", "on", "off"), default="auto",
                    help="after the TP phase, a short EP = world phase of --ep-model (config 5: DP attention, every "
                         "MoE layer an expert exchange over IPC peer memory across the devices), with a greedy-token "
                         "check against the dense fp32 EP = 1 model, reported as the 'ep' block.  auto: on when "
                         "world > 1")
    ap.add_argument("--ep-model", default="mixtral-8x7b")
    ap.add_argument("--ep-batch", type=int, default=256, help="concurrent requests PER RANK in the EP phase")
    ap.add_argument("--phase-child", choices=("tp", "ep"), default=None, help=argparse.SUPPRESS)
    ap.add_argument("--cr-ready-samples", type=int, default=3,
                    help="CR -> ready measurements with the predictor as a FRESH OS process (operator -> "
                         "ProcessLauncher -> /v2/health/ready), taken before the serving run on rank 0's GPU; "
                         "their median is p50_cr_ready_s.  0: report the in-process deploy time instead")
    return ap.parse_args(argv)


def _gpu_count() -> int:
    """Visible GPUs from the visible-devices env / the KFD topology in sysfs, never through HIP
    or torch (runtime/rank_launcher.py ``visible_gpu_count``): the launcher parent must not
    touch the GPU before its rank children exist, whatever torch's device count would do."""
    from mlopamd.runtime.rank_launcher import visible_gpu_count

    return visible_gpu_count()


def _http_check_on(a, world: int) -> bool:
    if a.http_check >= 0:
        return bool(a.http_check)
    return world == 1 and not a.no_operator and a.tp == 1 and a.ep == 1


def _process_ready(a, device_index: int | None, http: bool = False) -> dict:
    """Fresh predictor PROCESSES on one GPU, before this process touches HIP: p50 CR->ready over
    ``--cr-ready-samples`` of them, and with ``http`` the served rate of one more at this
    config under ``--batch`` closed-loop V2 HTTP clients (runtime/http_bench.py).  CPU: a
    float32 predictor without graphs (HTTP only when forced with ``--http-check 1``)."""
    import asyncio

    from mlopamd.runtime import http_bench

    env = {"MLOP_ENGINE_MAX_NUM_BATCHED_TOKENS": str(a.max_batched_tokens),
           "MLOP_ENGINE_MAX_MODEL_LEN": str(a.max_model_len)}
    if device_index is None:
        env.update({"MLOP_DEVICE": "cpu", "MLOP_DTYPE": "float32", "MLOP_ENGINE_USE_GRAPHS": "false",
                    "MLOP_ENGINE_NUM_KV_BLOCKS": "64", "OMP_NUM_THREADS": "2"})
    t0 = time.perf_counter()
    r = asyncio.run(http_bench.cr_ready_process(a.model, a.batch, env, samples=a.cr_ready_samples,
                                                gpus=[device_index] if device_index is not None else 8))
    r["probe_wall_s"] = round(time.perf_counter() - t0, 2)
    if http and (device_index is not None or a.http_check == 1):
        t0 = time.perf_counter()
        _progress(0, f"HTTP served-rate run: {a.batch} V2 clients against a fresh predictor process")
        h = http_bench.main(a, steps=max(a.steps, 40), warmup=a.warmup,
                            gpus=[device_index] if device_index is not None else 8,
                            extra_env=env if device_index is None else None)
        h["wall_s"] = round(time.perf_counter() - t0, 2)
        r["http"] = h
    return r


def launch(a, argv) -> int:
    """``--gpus N`` with no launcher around us: start N rank processes (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* in their env, LOCAL_RANK = the GPU index), wait for them, and exit
    with the first failing rank's status (the others are terminated).  Rank 0 prints the ONE
    JSON line.  Same pattern as the predictor's own ``--tp N`` (runtime/server.py launch_ranks)."""
    import signal
    import socket
    import subprocess

    n = a.gpus
    ngpu = _gpu_count()
    if ngpu and ngpu < n and not a.share_gpu:
        raise SystemExit(f"--gpus {n}: only {ngpu} GPUs visible")
    extra = {}
    if a.cr_ready_samples > 0 and not a.no_operator:
        extra["MLOP_BENCH_PROCESS_READY"] = json.dumps(_process_ready(a, 0 if ngpu else None,
                                                                      http=_http_check_on(a, n)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0",
                   MLOP_BENCH_LAUNCHER="1", **extra)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))

    def forward(sig, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(sig)

    signal.signal(signal.SIGTERM, forward)
    signal.signal(signal.SIGINT, forward)
    rc = 0
    try:
        while any(p.poll() is None for p in procs):
            bad = [p for p in procs if p.poll() not in (None, 0)]
            if bad:
                rc = bad[0].returncode
                break
            time.sleep(0.2)
        else:
            rc = next((p.returncode for p in procs if p.returncode), 0)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
                try:
                    p.wait(timeout=20)
                except subprocess.TimeoutExpired:
                    p.kill()
    return rc


def _apply_ab_ops(spec: str) -> dict:
    """``op=value,...`` -> torch.ops.mlop.<op>(value) for the in-process A/B switches
    (gemm_half_tile, gemm_big_variant, ...); returns each op's previous value."""
    from mlopamd import ops

    ops.load()
    prev = {}
    for item in filter(None, (t.strip() for t in spec.split(","))):
        name, _, val = item.partition("=")
        prev[name] = getattr(torch.ops.mlop, name)(int(val))
    return prev


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    a = parse(argv)
    if a.http:
        return http_main(a)
    if a.phase_child:
        return _phase_child_main(a)
    from mlopamd.parallel.comm import env_rank_info, init_distributed
    import torch.distributed as dist

    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(launch(a, argv))
    rank, local_rank, world = env_rank_info()
    if world != a.gpus:
        print(f"[bench] warning: --gpus {a.gpus} but WORLD_SIZE {world}: reporting the {world} ranks that ran",
              file=sys.stderr, flush=True)
    proc_ready = None
    if rank == 0 and a.cr_ready_samples > 0 and not a.no_operator:
        if os.environ.get("MLOP_BENCH_PROCESS_READY"):  # measured by our launcher parent
            proc_ready = json.loads(os.environ["MLOP_BENCH_PROCESS_READY"])
        else:  # before this process makes its first HIP call (the probe's predictor uses this GPU)
            proc_ready = _process_ready(a, local_rank if _gpu_count() else None, http=_http_check_on(a, world))
    if world > 1:
        init_distributed(backend="gloo" if a.share_gpu else None)
    dev = torch.device("cuda", 0 if a.share_gpu else local_rank) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    if a.ab_ops:
        _apply_ab_ops(a.ab_ops)

    from mlopamd.runtime.deploy import deploy_for_bench

    ekw = dict(max_num_seqs=a.batch, max_num_batched_tokens=a.max_batched_tokens,
               max_model_len=a.max_model_len, use_graphs=not a.no_graphs,
               prefill_min_batch=a.prefill_min_batch, max_decode_gap=a.max_decode_gap,
               mixed_prefill=not a.no_mixed, mixed_min_chunk=a.mixed_min_chunk,
               enable_prefix_caching=not a.no_prefix_cache, async_scheduling=not a.no_async)
    if a.kv_gb:
        ekw["kv_cache_bytes"] = int(a.kv_gb * 2**30)
    if a.share_gpu:
        os.environ.setdefault("MLOP_CUSTOM_AR", "force")  # K15 over the gloo group (same-GPU IPC)
    t0 = time.perf_counter()
    leader = True
    if a.ep > 1:
        assert a.tp == 1, "--ep with --tp: TP shards the experts itself"
        assert world % a.ep == 0, f"world {world} not divisible by --ep {a.ep}"
        from mlopamd.runtime.tp_worker import build_tp_engine

        engine, ps = build_tp_engine(a.model, 1, device=dev, seed=a.seed, engine_kwargs=ekw, ep=a.ep)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        ready_s = time.perf_counter() - t0
        deploy_info = {"path": "direct-ep", "ep": a.ep, "replicas": world // a.ep,
                       "weight_gb_per_gpu": round(engine.model.weight_bytes() / 1e9, 2),
                       "kv_blocks": engine.kv.num_blocks,
                       "exchange": "ipc" if getattr(ps.ep, "ex", None) is not None else "all_to_all"}
    elif a.tp > 1:
        assert world % a.tp == 0, f"world {world} not divisible by --tp {a.tp}"
        from mlopamd.runtime.tp_worker import build_tp_engine

        engine, ps = build_tp_engine(a.model, a.tp, device=dev, seed=a.seed + rank // a.tp, engine_kwargs=ekw)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        ready_s = time.perf_counter() - t0
        deploy_info = {"path": "direct-tp", "tp": a.tp, "replicas": world // a.tp,
                       "weight_gb_per_gpu": round(engine.model.weight_bytes() / 1e9, 2),
                       "kv_blocks": engine.kv.num_blocks}
        leader = ps.tp_rank == 0
    else:
        engine, ready_s, deploy_info = deploy_for_bench(
            model=a.model, device=dev, use_operator=not a.no_operator, seed=a.seed + rank, engine_kwargs=ekw)
    for k in ("model_build_ms", "kv_alloc_ms", "kv_malloc_ms", "kv_zero_ms", "graph_capture_ms"):  # start-up breakdown
        deploy_info[k] = engine.stats.get(k, 0)
    _progress(rank, f"engine ready in {ready_s:.1f} s (graph capture {engine.stats.get('graph_capture_ms', 0)} ms)")
    if not leader:  # TP worker: replay the leader's steps (and join its barriers) until STOP
        engine.worker_loop()
        _report(a, rank, world, dev, 0.0, 0.0, ready_s, {}, deploy_info, engine, None)
        dist.barrier()
        dist.destroy_process_group()
        return
    # steady-state serving is what the timed steps measure: let a lazily backed KV pool
    # finish its background fill first (CR->ready above is taken BEFORE this, when only
    # the first chunk is backed).  A partly backed pool admits fewer prompts, which turns
    # mixed steps into decode-only ones (29.9k vs 32.1k tok/s right after the GPU test suite)
    deploy_info.update(engine.kv.wait_ready())
    gen, elapsed, stats, ramp = serve_closed_loop(
        engine, a, a.batch, a.steps, a.warmup, rank,
        ep_group=engine.model.ps.ep_cpu if a.ep > 1 else None)
    deploy_info["ramp_steps"] = ramp
    if a.tp > 1:
        engine.shutdown()  # release the TP workers before the result gather
    res = _report(a, rank, world, dev, float(gen), elapsed, ready_s, stats, deploy_info, engine, proc_ready)
    if a.tp == 1:
        engine.shutdown()
    # the driver's N-GPU command is DP replicas; on the same GPUs, a short TP = N phase of Llama-3
    # (RCCL + the K15 IPC all-reduce across the N devices, with its own first-contact checks,
    # runtime/bench_tp.py) and an EP = N phase of Mixtral (the IPC expert exchange,
    # runtime/bench_ep.py) follow, reported as the line's "tp" / "ep" blocks.  They run in CHILD
    # processes (one per rank, their own process group): a first-contact failure there -- a hang,
    # an abort, a GPU fault -- ends the child, never this process, which holds the DP result and
    # prints the line either way
    phases = [ph for ph, on in (("tp", _tp_phase_on(a, world)), ("ep", _ep_phase_on(a, world))) if on]
    if phases:
        import gc

        del engine
        gc.collect()
        if dev.type == "cuda":  # the DP engines' memory back to the device for the children
            torch.cuda.synchronize(dev)
            torch.cuda.empty_cache()
        # the parents coordinate the phases over gloo (host only): a child that wedged the device
        # must not be able to hang the parent that holds the DP result
        coord = dist.new_group(backend="gloo") if world > 1 else None
        deadline = time.perf_counter() + a.phase_budget
        for ph in phases:
            blk = _phase_children(ph, a, argv, rank, world, coord, deadline)
            if res is not None:
                res[ph] = blk
    _emit(res)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _phase_children(phase: str, a, argv, rank: int, world: int, coord, deadline: float) -> dict | None:
    """Run ``runtime/bench_tp.tp_phase`` / ``runtime/bench_ep.ep_phase`` in one child process per
    rank (``--phase-child``), on a fresh rendezvous port, and collect rank 0's block from the
    file its child writes.  The phase gets min(``--tp-timeout``, what is left of
    ``--phase-budget``): the children's watchdog fires 15 s before the parents kill them.  The
    parents then meet at a barrier of ``coord`` (gloo); a child that died leaves ``error``."""
    import socket
    import subprocess
    import tempfile

    import torch.distributed as dist

    box = [None, None, deadline]
    if rank == 0:
        with socket.socket() as s_:
            s_.bind(("127.0.0.1", 0))
            box[0] = s_.getsockname()[1]
        fd, box[1] = tempfile.mkstemp(prefix=f"mlop-{phase}-phase-", suffix=".json")
        os.close(fd)
    if world > 1:
        dist.broadcast_object_list(box, src=0, group=coord)
    port, out_path, _ = box
    left = deadline - time.perf_counter()
    if world > 1:  # one verdict for the group (the clocks of the ranks differ slightly)
        t = torch.tensor([left], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=coord)
        left = float(t.item())
    child_limit = min(a.tp_timeout, left - 15.0)  # the child's own watchdog (it writes its error)
    limit = child_limit + 15.0                     # the parents kill it past this
    if left < 30:
        if rank == 0:
            try:
                os.unlink(out_path)
            except OSError:
                pass
            return {phase: world, "error": f"skipped: {max(left, 0):.0f} s left of --phase-budget {a.phase_budget:.0f}"}
        return None
    # the child is its own job: its own rendezvous (no torchrun agent store), same rank layout
    env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
               LOCAL_RANK=os.environ.get("LOCAL_RANK", str(rank)), MLOP_TP_PHASE_OUT=out_path,
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    # the child's own watchdog (--tp-timeout, the last occurrence wins) fires before the kill below
    cmd = [sys.executable, os.path.abspath(__file__), *argv, "--phase-child", phase,
           "--tp-timeout", f"{child_limit:.1f}"]
    t0 = time.perf_counter()
    _progress(rank, f"{phase.upper()} = {world} phase in a child process (port {port}, limit {limit:.0f} s)")
    p = subprocess.Popen(cmd, env=env)
    try:
        rc = p.wait(timeout=limit)
    except subprocess.TimeoutExpired:
        p.kill()
        try:
            rc = p.wait(timeout=20)
        except subprocess.TimeoutExpired:  # unkillable (stuck in the driver): leave it, report it
            rc = "unreaped"
        _progress(rank, f"{phase.upper()} phase child killed at its time limit")
    if world > 1:
        dist.barrier(group=coord)  # every child is gone (or given up on) before the parents go on
    if rank != 0:
        return None
    tp = None
    try:
        with open(out_path) as f:
            txt = f.read().strip()
        tp = json.loads(txt) if txt else None
    except (OSError, ValueError):
        tp = None
    finally:
        try:
            os.unlink(out_path)
        except OSError:
            pass
    if tp is None:
        tp = {phase: world, "error": f"{phase.upper()} phase child exited with {rc} and no result"}
    tp["child_rc"] = rc
    tp["child_wall_s"] = round(time.perf_counter() - t0, 2)
    tp["limit_s"] = round(limit, 1)
    return tp


def _phase_child_main(a) -> None:
    """``--phase-child tp|ep``: one rank of a parallel phase (spawned by ``_phase_children``);
    rank 0 writes the block, or the error that ended the phase, to $MLOP_TP_PHASE_OUT."""
    from mlopamd.parallel.comm import env_rank_info, init_distributed
    import torch.distributed as dist

    rank, local_rank, world = env_rank_info()
    out_path = os.environ.get("MLOP_TP_PHASE_OUT", "")
    phase = a.phase_child

    def write(block):
        if rank == 0 and out_path:
            with open(out_path, "w") as f:
                f.write(json.dumps(block))

    if a.share_gpu:
        os.environ.setdefault("MLOP_CUSTOM_AR", "force")  # K15 over the gloo group (same-GPU IPC)
    if world > 1:
        init_distributed(backend="gloo" if a.share_gpu else None)
    dev = torch.device("cuda", 0 if a.share_gpu else local_rank) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    if phase == "tp":
        from mlopamd.runtime.bench_tp import tp_phase as run_phase
    else:
        from mlopamd.runtime.bench_ep import ep_phase as run_phase
    block = run_phase(a, rank, world, dev, serve_closed_loop, lambda msg: write({phase: world, "error": msg}))
    write(block)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _ep_phase_on(a, world: int) -> bool:
    if a.ep_phase == "off" or a.tp > 1 or a.ep > 1:
        return False
    return world > 1 or a.ep_phase == "on"


def _tp_phase_on(a, world: int) -> bool:
    if a.tp_phase == "off" or a.tp > 1 or a.ep > 1:
        return False
    return world > 1 or a.tp_phase == "on"


_EMITTED = []


def _emit(res) -> None:
    """Rank 0 prints THE one JSON line (once, whichever of the normal end / the TP phase's
    watchdog gets there first)."""
    if res is None or _EMITTED:
        return
    _EMITTED.append(True)
    print(json.dumps(res), flush=True)


def serve_closed_loop(engine, a, batch, steps, warmup, rank, ep_group=None):
    """Closed-loop load: ``batch`` concurrent requests of ``--prompt-len`` random tokens and
    ``--output-len`` generated ones, the first cohort at staggered remaining lengths (steady-state
    age mix), each finished request replaced at once.  An untimed ramp admits and prefills the
    first cohort, then ``warmup`` untimed and ``steps`` timed engine steps bracketed by
    ``sync_point`` (device sync + world barrier, TP workers included).  Returns
    (generated tokens, seconds, step-stat deltas, ramp steps).  ``ep_group``: EP ranks step in
    lock-step, so the ramp continues while ANY rank still ramps."""
    from mlopamd.runtime.sampler import SamplingParams

    rng = np.random.default_rng(1234 + rank)
    V = engine.model.cfg.vocab_size
    P, O = a.prompt_len, a.output_len

    lo = min(1000, V // 4)
    shared = rng.integers(lo, V - lo, size=min(a.shared_prefix, P)).tolist()

    def new_request(max_tokens):
        prompt = shared + rng.integers(lo, V - lo, size=P - len(shared)).tolist()
        engine.add_request(prompt, SamplingParams(max_tokens=int(max_tokens), temperature=a.temperature,
                                                  top_k=50 if a.temperature > 0 else 0, ignore_eos=True))

    for i in range(batch):
        new_request(1 + (i * O) // batch)

    def run_steps(n):
        gen = 0
        for _ in range(n):
            outs = engine.step()
            gen += len(outs)
            for _ in outs.finished:
                new_request(O)
        return gen

    # ramp (untimed, not counted as warmup): the first cohort's prompts are all
    # admitted and prefilled, so the W warmup + K timed steps see the steady-state
    # mix (each step: every running sequence's decode token + the prompt chunks of
    # the requests that replaced the ones that finished) whatever W the caller picks
    ramp_cap = 4 * (batch * P) // max(1, a.max_batched_tokens) + 64
    ramp = 0
    backlog = max(a.prefill_min_batch, 2 * batch // max(1, O))  # ~2 steps of arrivals

    def ramp_more() -> bool:
        import torch.distributed as dist

        more = ramp < ramp_cap and (engine.stats["prefill_tokens"] < batch * P or len(engine.waiting) > backlog)
        if ep_group is not None:
            t = torch.tensor([int(more)], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=ep_group)
            more = bool(t.item())
        return more

    t_log = time.perf_counter()
    while a.ramp and ramp_more():
        run_steps(1)
        ramp += 1
        if time.perf_counter() - t_log > 20:  # a long ramp keeps saying it is alive
            t_log = time.perf_counter()
            _progress(rank, f"ramp step {ramp}: {engine.stats['prefill_tokens']} prompt tokens in, "
                            f"{len(engine.running)} running")
    _progress(rank, f"ramp done ({ramp} steps); {warmup} warmup + {steps} timed steps")
    run_steps(warmup)
    if not a.tune_in_timed:
        # shapes first seen from here on take the nearest tuned row count's GEMM backend
        # instead of being timed inside the measured steps
        from mlopamd import ops as _ops

        _ops.freeze_autotune()
    engine.sync_point()  # device sync + world barrier (TP workers join it)
    s0 = dict(engine.stats)
    t_start = time.perf_counter()
    gen = run_steps(steps)
    engine.sync_point()
    elapsed = time.perf_counter() - t_start
    stats = {k: engine.stats[k] - s0.get(k, 0) for k in engine.stats}
    return gen, elapsed, stats, ramp


def http_main(a):
    """bench.py --http: one replica, the whole serving path in the loop (see runtime/http_bench.py)."""
    from mlopamd.runtime import http_bench

    r = http_bench.main(a)
    res = {"metric": "served_tokens_per_sec", "value": r["served_tokens_per_sec_http"], "unit": "tokens/s",
           "n_gpus": 1, "steps": a.steps, "warmup": a.warmup, "ms_per_step": r["http_ms_per_step"],
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
           "data": "synthetic (random prompt tokens, random-init weights)",
           "config": {"model": "Llama-3-8B" if a.model == "llama3-8b" else a.model, "global_batch": a.batch,
                      "seq_len": a.prompt_len + a.output_len, "prompt_len": a.prompt_len,
                      "output_len": a.output_len, "parallelism": "dp1", "path": "http"},
           "p50_cr_ready_s": r["p50_cr_ready_process_s"], "http": r}
    print(json.dumps(res), flush=True)
    return res


def _progress(rank: int, msg: str) -> None:
    """One stderr line per phase (the JSON result line alone goes to stdout)."""
    print(f"[bench rank {rank}] {msg}", file=sys.stderr, flush=True)


def _report(a, rank, world, dev, gen, elapsed, ready_s, stats, deploy_info, engine, proc_ready=None):
    """Gather every rank's counts; rank 0 returns the result dict (the caller prints it)."""
    import torch.distributed as dist

    tot = torch.tensor([float(gen), elapsed, ready_s, float(stats.get("prefill_tokens", 0))], dtype=torch.float64)
    if world > 1:
        tt = tot.to(dev) if dev.type == "cuda" else tot
        gl = [torch.zeros_like(tt) for _ in range(world)]
        dist.all_gather(gl, tt)
        gathered = [g.cpu() for g in gl]
    else:
        gathered = [tot]
    total_gen = sum(float(g[0]) for g in gathered)
    max_t = max(float(g[1]) for g in gathered)
    readies = sorted(float(g[2]) for g in gathered if float(g[1]) > 0 or world == 1)
    p50_ready = readies[len(readies) // 2] if len(readies) % 2 else 0.5 * (readies[len(readies) // 2 - 1] + readies[len(readies) // 2])
    total_prefill = sum(float(g[3]) for g in gathered)
    value = total_gen / max_t
    if rank == 0:
        res = {
            "metric": "served_tokens_per_sec",
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000 * max_t / a.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (random prompt tokens, random-init weights)",
            "config": {"model": "Llama-3-8B" if a.model == "llama3-8b" else a.model,
                       "global_batch": a.batch * (world // a.tp), "seq_len": a.prompt_len + a.output_len,
                       "prompt_len": a.prompt_len, "output_len": a.output_len,
                       "parallelism": (f"dp{world // a.tp}" + (f"-tp{a.tp}" if a.tp > 1 else "")
                                       + (f"-ep{a.ep}" if a.ep > 1 else "")),
                       "shared_gpu": a.share_gpu,
                       "graphs": not a.no_graphs, "mixed_prefill": not a.no_mixed,
                       "async_scheduling": not a.no_async,
                       "prefill_min_batch": a.prefill_min_batch, "max_decode_gap": a.max_decode_gap,
                       "shared_prefix": a.shared_prefix, "prefix_cache": not a.no_prefix_cache},
            # CR -> ready with the predictor as a fresh OS process when measured (the honest
            # figure: process start + imports + HIP init inside); the in-process deploy time
            # (operator -> predictor built inside this already-running process) beside it
            "p50_cr_ready_s": (proc_ready["p50_cr_ready_process_s"] if proc_ready else round(p50_ready, 3)),
            "cr_ready_path": "fresh predictor process" if proc_ready else "in-process",
            "p50_cr_ready_in_process_s": round(p50_ready, 3),
            "cr_ready_process": proc_ready,
            # the same config served over V2 HTTP by a fresh predictor process (operator ->
            # ProcessLauncher -> Router -> aiohttp clients), measured before the engine-direct run
            "served_tokens_per_sec_http": ((proc_ready or {}).get("http") or {}).get("served_tokens_per_sec_http"),
            "served_tokens_per_sec_per_gpu": round(value / world, 2),
            "per_rank_tokens_per_sec": [round(float(g[0]) / float(g[1]), 2) if float(g[1]) > 0 else 0.0
                                        for g in gathered],
            "dist": {"world_size": world, "backend": dist.get_backend() if dist.is_initialized() else None,
                     "launcher": "bench.py" if os.environ.get("MLOP_BENCH_LAUNCHER") else
                     ("torch.distributed.run" if "TORCHELASTIC_RUN_ID" in os.environ else
                      ("external" if world > 1 else "none"))},
            "prefill_tokens_per_sec": round(total_prefill / max_t, 2),
            "step_mix": stats,
            "deploy": deploy_info,
        }
        try:
            from mlopamd import ops

            # backend that actually RAN per projection shape (eager calls and graph captures of
            # this process), and the configured mode
            res["gemm_backend"] = ops.gemm_used()
            res["gemm_mode"] = ops.GEMM_BACKEND
        except Exception:  # noqa: BLE001
            pass
        if a.save_gemm_table:
            from mlopamd import ops

            ops.save_gemm_table(a.save_gemm_table)
        return res
    return None


if __name__ == "__main__":
    main()
