#!/bin/bash
# grouped <= 32-rows-per-expert rule: numerics, then Mixtral batch 32 / 64 A/B
source scripts/gpu_check.sh
step moe_tests 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "moe or mixtral or grouped"
for b in 32 64; do
  for i in 1 2; do
    step "n${b}_on$i" 300 python3 bench.py --no-operator --model mixtral-8x7b --batch $b --steps 30 --warmup 10 --cr-ready-samples 0
    step "n${b}_off$i" 300 python3 bench.py --no-operator --model mixtral-8x7b --batch $b --steps 30 --warmup 10 --cr-ready-samples 0 --ab-ops gemm_grouped_narrow=0
  done
done
