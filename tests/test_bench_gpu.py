"""The driver's N-GPU bench command on hardware, rehearsed on one MI355X: ``bench.py --gpus 2
--share-gpu`` (both ranks on cuda:0 over gloo, K15 forced over same-GPU IPC) with tiny models.
The line must carry the DP value and both extra phases from their child processes: the TP
phase with K15's start-up self-check passed and the greedy tokens inside the dense fp32
oracle's bound, the EP phase with the IPC expert exchange and tokens equal to an EP = 1
engine's (runtime/bench_tp.py, runtime/bench_ep.py, profiles/r06_tp_phase.md)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_share_gpu_tp_ep_phases():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--share-gpu", "--kv-gb", "4",
           "--model", "tiny-llama", "--batch", "16", "--steps", "4", "--warmup", "2", "--cr-ready-samples", "0",
           "--tp-batch", "16", "--tp-steps", "3", "--tp-warmup", "1", "--ep-model", "tiny-mixtral",
           "--ep-batch", "16", "--phase-budget", "200"]
    r = subprocess.run(cmd, cwd="/tmp", capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0
    tp, ep = d["tp"], d["ep"]
    assert tp["child_rc"] == 0 and "error" not in tp, tp
    assert tp["k15"] == "ok" and all(tp["k15_check"]["checks"].values()) and tp["k15_error_word"] == 0
    assert tp["first_token_match"] and tp["tokens_match"] and tp["tokens_per_sec"] > 0
    assert ep["child_rc"] == 0 and "error" not in ep, ep
    assert ep["exchange"] == "ipc" and ep["tokens_match"] and ep["tokens_equal_ep1_engine"] == ep["tokens_checked"]
    assert ep["tokens_per_sec"] > 0
