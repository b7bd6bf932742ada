#!/bin/bash
# small-M O -> gate_up without the add + RMSNorm launch: numerics, then Llama batch 16 / 32 / 64 A/B
source scripts/gpu_check.sh
step tests 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_norm_chain_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py -k "small or gemm or model or decode or norm"
for b in 16 32 64; do
  for i in 1 2; do
    step "sf${b}_on$i" 300 python3 bench.py --no-operator --batch $b --steps 60 --warmup 10 --cr-ready-samples 0
    step "sf${b}_off$i" 300 python3 bench.py --no-operator --batch $b --steps 60 --warmup 10 --cr-ready-samples 0 --ab-ops gemm_small_fused=0
  done
done
