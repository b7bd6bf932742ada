#!/bin/bash
# Stream-K tail of the ping-pong GEMM: numerics first, then the projection A/B (SK on) and
# the same with SK off, then the headline bench.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_sk 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "stream_k or qkv_rope_cache_fused or test_gemm or moe_pipeline or grouped"
step proj_sk 300 env BENCH_MS=2040,2304,3072,4088,4352,6144 python scripts/bench_proj.py
step proj_dp 300 env MLOP_GEMM_SK=0 BENCH_MS=2040,2304,3072,4088,4352,6144 python scripts/bench_proj.py
