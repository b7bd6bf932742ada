"""Cost of the in-serving kernel-time sampler (runtime/gpu_metrics.py KernelTimeSampler) on the
engine thread: the step loop of runtime/backends.py (before_step / engine.step / after_step) under a
closed-loop Llama-3-8B load, sampler OFF vs ON (period ``--period`` s), interleaved ``--rounds``
times, ``--seconds`` of serving each.  Reports step-time p50 / p99 / max per mode, every window's
engine-thread cost (open + close + reduce) and the one-time tracer start-up (``warm``), which a
fresh sampler pays inside its first window unless ``warm`` ran first (``--no-warm`` shows that).

Usage (GPU box): python scripts/bench_ktime.py [--batch 256] [--seconds 30] [--period 5] [--rounds 2]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--output-len", type=int, default=256)
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--period", type=float, default=5.0)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--no-warm", action="store_true")
    ap.add_argument("--sync-reduce", action="store_true", help="reduce the window on the engine thread")
    a = ap.parse_args()

    from mlopamd.runtime.deploy import build_engine
    from mlopamd.runtime.gpu_metrics import KernelTimeSampler
    from mlopamd.runtime.sampler import SamplingParams

    dev = torch.device("cuda", 0)
    eng = build_engine(a.model, device=dev, max_num_seqs=a.batch, max_num_batched_tokens=8192,
                       max_model_len=a.prompt_len + a.output_len + 64)
    rng = np.random.default_rng(0)
    V = eng.model.cfg.vocab_size

    def add(n_out):
        eng.add_request(rng.integers(1000, V - 1000, size=a.prompt_len).tolist(),
                        SamplingParams(max_tokens=int(n_out), ignore_eos=True))

    for i in range(a.batch):
        add(1 + (i * a.output_len) // a.batch)

    def serve(seconds, sampler):
        times = []
        t_end = time.perf_counter() + seconds
        while time.perf_counter() < t_end:
            t0 = time.perf_counter()
            if sampler is not None:
                sampler.before_step(t0)
            outs = eng.step()
            now = time.perf_counter()
            if sampler is not None:
                sampler.after_step(now)
            for _ in outs.finished:
                add(a.output_len)
            times.append(1e3 * (time.perf_counter() - t0))
        return times

    serve(10.0, None)  # ramp: every first-cohort prompt admitted, steady mix
    res = {"config": vars(a), "off": [], "on": []}
    sampler = KernelTimeSampler(period_s=a.period, async_reduce=not a.sync_reduce)
    warm_steps = []
    if not a.no_warm:  # as the predictor does: in the background, while serving
        sampler.warm(background=True)
        t_w = time.perf_counter()
        while sampler._warm_thread.is_alive():
            warm_steps += serve(0.05, None)
        res["warm_wall_ms"] = round(1e3 * (time.perf_counter() - t_w), 1)
    res["warm_ms"] = sampler.warm_ms
    for r in range(a.rounds):
        res["off"] += serve(a.seconds, None)
        sampler._next = time.perf_counter() + 0.5  # first window half a second into the run
        sampler.join()
        res["on"] += serve(a.seconds, sampler)
        print(f"round {r + 1}: off {len(res['off'])} steps, on {len(res['on'])} steps, "
              f"windows {sampler.windows}", file=sys.stderr, flush=True)
    sampler.join()
    if warm_steps:
        w = np.asarray(warm_steps)
        res["during_warm"] = {"steps": int(w.size), "p50_ms": round(float(np.percentile(w, 50)), 3),
                              "max_ms": round(float(w.max()), 3)}
    out = {"warm_ms": res["warm_ms"], "warm_wall_ms": res.get("warm_wall_ms"), "during_warm": res.get("during_warm"),
           "async_reduce": sampler.async_reduce, "reduce_ms": sampler.reduce_ms,
           "windows": sampler.windows, "window_host_ms": sampler.host_ms,
           "last_shares": {k: round(v, 4) for k, v in sorted(sampler.last.items(), key=lambda kv: -kv[1])[:8]}}
    for mode in ("off", "on"):
        t = np.asarray(res[mode])
        out[mode] = {"steps": int(t.size), "p50_ms": round(float(np.percentile(t, 50)), 3),
                     "p99_ms": round(float(np.percentile(t, 99)), 3), "max_ms": round(float(t.max()), 3),
                     "mean_ms": round(float(t.mean()), 3)}
    out["p99_on_over_off"] = round(out["on"]["p99_ms"] / out["off"]["p99_ms"], 4)
    out["config"] = res["config"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
