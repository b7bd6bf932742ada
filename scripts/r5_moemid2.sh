#!/bin/bash
# mid dispatch over prefill-sized T too: numerics, then Mixtral A/B of the token range
# (16384 = default, 1024 = the first version, 16 = off)
source scripts/gpu_check.sh
step moe_tests 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "moe or mixtral or grouped"
for b in 256 1024; do
  for i in 1 2; do
    step "m${b}_all$i" 300 python3 bench.py --no-operator --model mixtral-8x7b --batch $b --steps 30 --warmup 10 --cr-ready-samples 0
    step "m${b}_1k$i" 300 python3 bench.py --no-operator --model mixtral-8x7b --batch $b --steps 30 --warmup 10 --cr-ready-samples 0 --ab-ops moe_mid_max_tokens=1024
    step "m${b}_off$i" 300 python3 bench.py --no-operator --model mixtral-8x7b --batch $b --steps 30 --warmup 10 --cr-ready-samples 0 --ab-ops moe_mid_max_tokens=16
  done
done
