#!/bin/bash
# ADVICE fixes (padded-row zero store in the fused split-KV combine, GEMV KW4 env) +
# hand-written GEMM vs hipBLASLt at the headline's mixed-step M.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_attn 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "paged_attention or gemv or flash"
BENCH_MS=2048,3072,3840,4096 step gemm_big 300 python scripts/bench_gemm.py
