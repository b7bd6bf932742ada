#!/bin/bash
# Half-height four-wave tile (planner variant 6): numerics, the mid-M sweep with the planner's
# choice, and interleaved serving A/Bs at batch 512 / 1024 / 2048 (profiles/r05_gemm_w4h.md).
source scripts/gpu_check.sh
step w4h_tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_w4_gpu.py \
  tests/test_norm_chain_gpu.py tests/test_kernels_gpu.py -k "gemm or w4 or chain"
step w4h_midm 400 python -u scripts/bench_mid_m.py --ms 384,640,768,896,1152,1280,1408,1792,2304 --shapes qkv,o,down
for b in 512 1024; do
  for i in 1 2; do
    step "ab_b${b}_on$i" 400 python3 bench.py --steps 30 --warmup 8 --cr-ready-samples 0 --http-check 0 --batch $b
    step "ab_b${b}_off$i" 400 python3 bench.py --steps 30 --warmup 8 --cr-ready-samples 0 --http-check 0 --batch $b --ab-ops gemm_half_tile=0
  done
done
step ab_b2048_on 400 python3 bench.py --steps 30 --warmup 8 --cr-ready-samples 0 --http-check 0
step ab_b2048_off 400 python3 bench.py --steps 30 --warmup 8 --cr-ready-samples 0 --http-check 0 --ab-ops gemm_half_tile=0
