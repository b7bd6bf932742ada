#!/bin/bash
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step w4tests 300 python -u -m pytest tests/test_gemm_w4_gpu.py -x -q --timeout 120 --timeout-method thread
step w4sched 400 env BENCH_VARIANTS=5 BENCH_W4_SCHEDS=0,1,2 BENCH_MS=4088,2048 python -u scripts/bench_bigm.py
