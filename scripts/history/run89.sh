#!/bin/bash
# Ping-pong + stream-K for launches of <= 128 tiles (o / down at M = 1024 .. 2048): numerics,
# then the projection A/B with stream-K on / off.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_sk 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "stream_k or qkv_rope_cache_fused or test_gemm or moe_pipeline or grouped"
step proj_sk 300 env BENCH_MS=1024,1536,2040,2048 python scripts/bench_proj.py
step proj_dp 300 env MLOP_GEMM_SK=0 BENCH_MS=1024,1536,2040,2048 python scripts/bench_proj.py
