#!/bin/bash
# hand-written (default) vs the per-shape library table (MLOP_GEMM_BACKEND=auto)
# at batch 512 / 768, interleaved, plus the mid-M sweep of the planner and the headline A/B of
# the half-height tile (profiles/r05_gemm_w4h.md).
source scripts/gpu_check.sh
step midm 300 python -u scripts/bench_mid_m.py --ms 384,512,640,1024,1152,1408,2048 --shapes qkv,o,down
for b in 512 768; do
  for i in 1 2; do
    step "b${b}_mlop$i" 400 python3 bench.py --steps 60 --warmup 10 --no-operator --batch $b
    step "b${b}_auto$i" 400 env MLOP_GEMM_BACKEND=auto python3 bench.py --steps 60 --warmup 10 --no-operator --batch $b
  done
done
for i in 1 2; do
  step "head_on$i" 400 python3 bench.py --steps 20 --warmup 5 --cr-ready-samples 0 --http-check 0
  step "head_off$i" 400 python3 bench.py --steps 20 --warmup 5 --cr-ready-samples 0 --http-check 0 --ab-ops gemm_half_tile=0
done
