#!/bin/bash
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step w4tests 300 python -u -m pytest tests/test_gemm_w4_gpu.py tests/test_races_gpu.py -x -q --timeout 120 --timeout-method thread
step w4ab 300 env BENCH_VARIANTS=3,5 BENCH_MS=4088,2048 python -u scripts/bench_bigm.py
step ksweep 400 python -u scripts/bench_w4_k.py
