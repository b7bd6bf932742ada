#!/bin/bash
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step tests 600 python -u -m pytest tests/test_gemm_w4_gpu.py tests/test_kernels_gpu.py -x -q -k "silu or gemm or gemv" --timeout 120 --timeout-method thread
step w4ab 300 env BENCH_VARIANTS=3,5 BENCH_MS=4088,2048 python -u scripts/bench_bigm.py
