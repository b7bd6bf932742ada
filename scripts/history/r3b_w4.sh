#!/bin/bash
# Four-wave asm GEMM (variant 5): numerics first, then the A/B vs ping-pong and hipBLASLt.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step w4tests 300 python -u -m pytest tests/test_gemm_w4_gpu.py -x -v --timeout 120 --timeout-method thread
step w4ab 300 env BENCH_VARIANTS=3,5 BENCH_MS=4096,4088,2048 python -u scripts/bench_bigm.py
