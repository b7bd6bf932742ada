#!/bin/bash
# small-M O-projection rule (one K range, narrow tiles): numerics, then serving A/B at batch 16/32/64
source scripts/gpu_check.sh
step tests 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "gemm or norm or model or decode"
for b in 16 32 64; do
  for i in 1 2; do
    step "ab_b${b}_on$i" 300 python3 bench.py --no-operator --batch $b --steps 60 --warmup 10 --cr-ready-samples 0
    step "ab_b${b}_off$i" 300 python3 bench.py --no-operator --batch $b --steps 60 --warmup 10 --cr-ready-samples 0 --ab-ops gemm_small_nosplit=0
  done
done
