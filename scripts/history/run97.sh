#!/bin/bash
# Fused QKV + RoPE GEMM with the V-head tiles dispatched first: numerics + projection A/B
# (compare qkv rows with scripts/run87.sh / run96.sh: fused 217-229 us at M=4088).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_rope 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "qkv_rope or rope_cache or stream_k"
step proj 300 env BENCH_MS=2040,3072,4088,6144,8192 python scripts/bench_proj.py
