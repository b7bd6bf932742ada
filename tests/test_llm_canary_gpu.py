"""BASELINE configs 3 and 5 on one MI355X: the operator canaries a new version of
an LLM predictor whose pods are real runtime processes on the GPU (HIP kernels,
hipGraph decode), gated on the Seldon-executor metrics they export plus the
TPOT guard; a regressed new version (injected into its pods only) must be
rolled back automatically, a healthy one promoted (controller/llm_demo.py)."""
import asyncio

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("arch,regress,expect", [
    ("tiny-llama", None, "Promoted"),
    ("tiny-llama", "latency", "RolledBack"),
    ("tiny-mixtral", "errors", "RolledBack"),
    # v2 slowed on the device only; p95 / mean latency may rise 10x and still
    # pass, so the rollback must come from the GPU-side TPOT guard at its 1.10 default
    ("tiny-llama", "tpot", "RolledBack"),
])
def test_llm_canary_on_gpu(gpu, arch, regress, expect):
    from mlopamd.controller.llm_demo import run_llm_canary

    r = asyncio.run(run_llm_canary(arch, regress, "cuda", concurrency=8, max_tokens=16, timeout_s=300))
    assert r["canary_phase"] == expect, r
    assert r["served"] > 0 and r["by_predictor"].get("v2", 0) > 0
    if expect == "RolledBack":
        assert r["final_predictors"] == {"v1": 100} and r["rolled_back_version"] == "2"
        assert r["events"][-1] == "RollbackComplete"
        if regress == "tpot":  # the guard that decided is named in status.error
            assert "tpot_avg" in (r["error"] or ""), r
            assert not any(k in (r["error"] or "") for k in ("latency_95th", "latency_avg", "error_rate")), r
    else:
        assert r["final_predictors"] == {"v2": 100} and r["events"][-1] == "PromotionComplete"
