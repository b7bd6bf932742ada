#!/bin/bash
# Mixtral-8x7B mid batches: grouped (MoE) 64-row tiles on narrow N with a 6-deep ring vs 3.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step moe_tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 150 --timeout-method thread -k "grouped or moe"
for r in 1 2; do
  for b in 32 64; do
    step mx_s3_${b}_$r 300 env MLOP_GEMM_GROUPED_SMALL_STAGES=3 python bench.py --model mixtral-8x7b --batch $b --steps 60 --warmup 20 --no-operator
    step mx_s6_${b}_$r 300 python bench.py --model mixtral-8x7b --batch $b --steps 60 --warmup 20 --no-operator
  done
done
