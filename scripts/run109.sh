#!/bin/bash
# Split-K grouped GEMM for mid-size MoE batches: numerics, then Mixtral at batch 64 / 256
# (before: 3,032 / 7,593 tok/s, scripts/run108.sh).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_moe 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread -k "moe or grouped or mixtral"
step mix_b64 600 python bench.py --model mixtral-8x7b --batch 64 --steps 60 --warmup 20 --no-operator
step mix_b256 600 python bench.py --model mixtral-8x7b --batch 256 --steps 60 --warmup 20 --no-operator
step mix_b64_nosk 600 env MLOP_GEMM_SK=0 python bench.py --model mixtral-8x7b --batch 64 --steps 60 --warmup 20 --no-operator
