#!/bin/bash
# MoE dispatch with the post-attention add + RMSNorm prologue: kernel / model tests, then
# Mixtral decode benches at batch 1 and 4 (before: 203.8 / 321 tok/s, run78).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_moe 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread -k "moe or mixtral"
step mix_b1 400 python bench.py --model mixtral-8x7b --batch 1 --steps 100 --warmup 10 --no-operator
step mix_b4 400 python bench.py --model mixtral-8x7b --batch 4 --steps 100 --warmup 10 --no-operator
