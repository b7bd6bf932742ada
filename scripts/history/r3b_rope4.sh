#!/bin/bash
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step w4tests 300 python -u -m pytest tests/test_gemm_w4_gpu.py tests/test_races_gpu.py -x -q --timeout 120 --timeout-method thread
step kern 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "rope or gemm" --timeout 120 --timeout-method thread
step rope_var 300 python -u scripts/bench_rope_var.py
