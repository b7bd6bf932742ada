#!/bin/bash
# NOTE: gemm4.hip (the four-wave kernel) was removed after this run: profiles/r02_gemm_fourwave_rejected.md
# Four-wave 256x256 GEMM (gemm4.hip): numerics, then A/B vs the ping-pong kernel and hipBLASLt.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_w4 300 python -u -m pytest tests/test_gemm4_gpu.py -x -q --timeout 120 --timeout-method thread
step bench_w4 400 python scripts/bench_gemm4.py
