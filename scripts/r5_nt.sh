#!/bin/bash
# non-temporal weight loads in the one-m-tile small-M / grouped decode GEMMs (gemm_small_nt):
# numerics with nt on, cold-weight microbench, then Llama batch 16 / 64 and Mixtral batch 64 A/B
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step micro 300 python3 scripts/bench_small_m.py --nt --ms 16,64
for i in 1 2; do
  for b in 16 64; do
    step "l${b}_off$i" 300 python3 bench.py --no-operator --batch $b --steps 60 --warmup 10 --cr-ready-samples 0
    step "l${b}_on$i" 300 python3 bench.py --no-operator --batch $b --steps 60 --warmup 10 --cr-ready-samples 0 --ab-ops gemm_small_nt=3
  done
  step "m64_off$i" 300 python3 bench.py --no-operator --model mixtral-8x7b --batch 64 --steps 30 --warmup 10 --cr-ready-samples 0
  step "m64_on$i" 300 python3 bench.py --no-operator --model mixtral-8x7b --batch 64 --steps 30 --warmup 10 --cr-ready-samples 0 --ab-ops gemm_small_nt=3
done
