"""bench.py contract on CPU: the driver's JSON line, single process and 2 ranks over
gloo (torch.distributed.run, 127.0.0.1), tiny Llama shapes through the same
operator-deploy + engine path as the MI355X run."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config"}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(cmd):
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, cwd="/tmp", capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # exactly one JSON line (rank 0)
    return json.loads(lines[0])


ARGS = ["--model", "tiny-llama", "--steps", "4", "--warmup", "2", "--batch", "8"]
TP_ARGS = ["--tp-batch", "16", "--tp-steps", "3", "--tp-warmup", "1", "--ep-model", "tiny-mixtral", "--ep-batch", "8"]


def test_bench_single_process_json():
    d = _run([sys.executable, os.path.join(ROOT, "bench.py"), *ARGS])
    assert KEYS <= set(d)
    assert d["n_gpus"] == 1 and d["steps"] == 4 and d["warmup"] == 2 and d["value"] > 0
    assert d["config"]["parallelism"] == "dp1" and d["higher_is_better"] is True
    assert d["deploy"]["path"] == "operator" and d["p50_cr_ready_s"] > 0
    # CR -> ready measured with the predictor as a fresh OS process
    assert d["cr_ready_path"] == "fresh predictor process"
    assert d["p50_cr_ready_s"] == d["cr_ready_process"]["p50_cr_ready_process_s"]
    assert max(d["cr_ready_process"]["cr_ready_process_samples_s"]) >= \
        d["cr_ready_process"]["predictor_process_ready_s"] > 0
    # a median of three fresh processes
    samples = d["cr_ready_process"]["cr_ready_process_samples_s"]
    assert len(samples) == 3 and d["p50_cr_ready_s"] == sorted(samples)[1]
    assert "served_tokens_per_sec_http" in d  # None on CPU unless forced (below)


def test_bench_reports_http_served_rate():
    """``--http-check 1``: the default line also carries the HTTP-served rate of the same config
    (fresh predictor process, operator + Router + V2 clients) measured before the engine run."""
    d = _run([sys.executable, os.path.join(ROOT, "bench.py"), "--http-check", "1", "--cr-ready-samples", "1",
              *ARGS])
    h = d["cr_ready_process"]["http"]
    assert d["served_tokens_per_sec_http"] == h["served_tokens_per_sec_http"] > 0
    assert h["http_errors"] == 0 and h["http_window_steps"] >= 40 and d["value"] > 0


def test_bench_two_ranks_gloo():
    d = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
              "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
              os.path.join(ROOT, "bench.py"), "--gpus", "2", "--cr-ready-samples", "0", *ARGS, *TP_ARGS])
    assert d["dist"] == {"world_size": 2, "backend": "gloo", "launcher": "torch.distributed.run"}
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["config"]["global_batch"] == 16 and d["value"] > 0
    # whole-job aggregate over ranks = per-GPU value x N
    assert abs(d["served_tokens_per_sec_per_gpu"] * 2 - d["value"]) < 1e-3 * d["value"] + 0.02
    # after the DP replicas, a TP = world phase on the same ranks (the
    # xGMI path on a GPU node): its own rate, K15 state (off on CPU) and the greedy tokens of
    # 8 fixed prompts against the dense TP = 1 recompute
    tp = d["tp"]
    assert tp["tp"] == 2 and tp["world"] == 2 and tp["backend"] == "gloo" and tp["k15"] == "off"
    assert tp["tokens_per_sec"] > 0 and tp["steps"] == 3 and tp["batch"] == 16
    assert tp["first_token_match"] and tp["tokens_match"] and tp["tokens_checked"] == 32
    assert tp["child_rc"] == 0  # the phase ran in child processes (bench.py --phase-child tp)
    # and an EP = world phase of a MoE model: DP attention + the expert exchange, greedy tokens
    # against the dense fp32 EP = 1 model whose experts are the group's
    ep = d["ep"]
    assert ep["ep"] == 2 and ep["model"] == "tiny-mixtral" and ep["exchange"] == "all_to_all"
    assert ep["tokens_per_sec"] > 0 and ep["child_rc"] == 0
    assert ep["first_token_match"] and ep["tokens_match"] and ep["tokens_checked"] == 16
    assert ep["tokens_equal_ep1_engine"] == 16 and ep["check_layers"] == 2


def test_bench_tp_phase_watchdog_keeps_the_dp_result():
    """A TP phase that overruns --tp-timeout (a first-contact hang on real peers) must not cost
    the DP value: rank 0 prints THE line with tp.error and every rank exits 0."""
    d = _run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--cr-ready-samples", "0",
              *ARGS, "--tp-batch", "64", "--tp-steps", "200", "--tp-timeout", "3", "--ep-phase", "off"])
    assert d["value"] > 0 and d["n_gpus"] == 2
    assert "tp-timeout" in d["tp"]["error"] and d["tp"]["child_rc"] == 3


def test_bench_phase_budget_skips_what_does_not_fit():
    """The TP and EP phases share ``--phase-budget``: a hang in the first cannot push the command
    past the driver's limit.  With less than 30 s of budget, both say so and do not start."""
    d = _run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--cr-ready-samples", "0",
              *ARGS, *TP_ARGS, "--phase-budget", "25"])
    assert d["value"] > 0 and d["n_gpus"] == 2
    assert d["tp"]["error"].startswith("skipped") and d["ep"]["error"].startswith("skipped")


def test_bench_tp_phase_child_crash_keeps_the_dp_result():
    """A rank of the TP phase that dies outright (abort: what a GPU fault does to a process) ends
    only its child process: the DP ranks still print THE line, with tp.error, and exit 0."""
    env = dict(os.environ, OMP_NUM_THREADS="2", MLOP_INJECT_TP_PHASE_ABORT="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--cr-ready-samples", "0",
                        *ARGS, *TP_ARGS, "--tp-timeout", "20", "--ep-phase", "off"], cwd="/tmp",
                       capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["value"] > 0 and "no result" in d["tp"]["error"] and d["tp"]["child_rc"] != 0


def test_bench_self_launches_n_ranks():
    """``python bench.py --gpus 2`` with no torchrun around it (the driver's plain command):
    bench.py launches the 2 rank processes itself, both replicas' tokens are counted, and
    the line says which world actually ran."""
    d = _run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *ARGS, *TP_ARGS])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["tp"]["tokens_per_sec"] > 0 and d["tp"]["first_token_match"]
    assert d["dist"] == {"world_size": 2, "backend": "gloo", "launcher": "bench.py"}
    assert len(d["per_rank_tokens_per_sec"]) == 2 and min(d["per_rank_tokens_per_sec"]) > 0
    assert d["cr_ready_path"] == "fresh predictor process"  # probed once by the launcher parent


def test_bench_self_launches_tp_group():
    """``bench.py --gpus 2 --tp 2``: one TP=2 replica over the 2 self-launched ranks."""
    d = _run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--tp", "2",
              "--cr-ready-samples", "0", *ARGS])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp1-tp2" and d["value"] > 0
    assert d["config"]["global_batch"] == 8 and d["deploy"]["tp"] == 2
    assert d["dist"]["world_size"] == 2 and d["dist"]["launcher"] == "bench.py"


def test_bench_expert_parallel_mode():
    """``bench.py --gpus 2 --ep 2 --model tiny-mixtral`` (config 5): two DP-attention engines in
    lock-step, every MoE layer an expert exchange (gloo all_to_all on CPU, the IPC exchange on
    GPU); both ranks' tokens counted."""
    d = _run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--ep", "2", "--model", "tiny-mixtral",
              "--steps", "4", "--warmup", "2", "--batch", "8", "--cr-ready-samples", "0"])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2-ep2" and d["deploy"]["ep"] == 2
    assert d["deploy"]["exchange"] == "all_to_all" and min(d["per_rank_tokens_per_sec"]) > 0


def test_deploy_fails_fast_when_predictor_cannot_start():
    """A predictor whose start-up raises (here: a 1-page KV cache) fails the bench's
    operator deploy at once, not after the 900 s readiness timeout."""
    import time

    import pytest

    sys.path.insert(0, ROOT)
    from mlopamd.controller.local import deploy_and_wait

    t0 = time.time()
    with pytest.raises(RuntimeError, match="failed to start"):
        deploy_and_wait(model="tiny-llama", device="cpu", timeout_s=120.0,
                        engine_kwargs=dict(num_kv_blocks=1, use_graphs=False))
    assert time.time() - t0 < 60


def test_http_bench_end_to_end_on_cpu():
    """bench.py --http's driver on a tiny model: CR -> operator -> SD -> a fresh predictor
    process (ProcessLauncher, container command) -> closed-loop V2 /generate clients through
    the Router; the window is counted in the predictor's own engine steps."""
    import asyncio

    from mlopamd.runtime import http_bench

    r = asyncio.run(http_bench.run(
        "tiny-llama", batch=8, prompt_len=16, output_len=8, steps=10, warmup=3, ready_timeout_s=180,
        ramp_timeout_s=60, engine_env={"MLOP_DEVICE": "cpu", "MLOP_DTYPE": "float32", "MLOP_ENGINE_USE_GRAPHS": "false",
                                       "MLOP_ENGINE_NUM_KV_BLOCKS": "64", "MLOP_ENGINE_MAX_MODEL_LEN": "128",
                                       "OMP_NUM_THREADS": "2"}))
    assert r["http_window_steps"] >= 10 and r["served_tokens_per_sec_http"] > 0 and r["http_errors"] == 0
    assert r["p50_cr_ready_process_s"] >= r["predictor_process_ready_s"] > 0
