#!/bin/bash
# Grouped (MoE) GEMM with the on-device planned stream-K tail: numerics, then Mixtral at
# concurrency 1024 (before: 16,187 tok/s, scripts/run94.sh) with stream-K on / off.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_sk 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "stream_k or grouped or moe or test_gemm"
step mix_b1024 600 python bench.py --model mixtral-8x7b --batch 1024 --steps 60 --warmup 20 --no-operator
step mix_b1024_nosk 600 env MLOP_GEMM_SK=0 python bench.py --model mixtral-8x7b --batch 1024 --steps 60 --warmup 20 --no-operator
