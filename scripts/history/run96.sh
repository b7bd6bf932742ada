#!/bin/bash
# Dead-quadrant MFMA skip (ragged last m-tiles, MoE experts' last m-tiles): numerics, the
# projection A/B at ragged and full M, and Mixtral at concurrency 1024, skip on / off.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_sk 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "stream_k or grouped or moe or test_gemm or qkv_rope"
step proj_skip 300 env BENCH_MS=2040,2100,4088,4160 python scripts/bench_proj.py
step proj_noskip 300 env MLOP_GEMM_SKIP_DEAD=0 BENCH_MS=2040,2100,4088,4160 python scripts/bench_proj.py
step mix_skip 600 python bench.py --model mixtral-8x7b --batch 1024 --steps 60 --warmup 20 --no-operator
step mix_noskip 600 env MLOP_GEMM_SKIP_DEAD=0 python bench.py --model mixtral-8x7b --batch 1024 --steps 60 --warmup 20 --no-operator
