#!/bin/bash
# small-batch check of the non-temporal defaults: all off vs defaults, batch 1 / 4 / 16
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  for b in 1 4 16; do
    step "b${b}_off$i" 300 python3 bench.py --no-operator --batch $b --steps 40 --warmup 10 --cr-ready-samples 0 --ab-ops attn_kv_nt=0,gemm_slab_nt=0,gemm_small_nt=0
    step "b${b}_att0_$i" 300 python3 bench.py --no-operator --batch $b --steps 40 --warmup 10 --cr-ready-samples 0 --ab-ops attn_kv_nt=0
    step "b${b}_on$i" 300 python3 bench.py --no-operator --batch $b --steps 40 --warmup 10 --cr-ready-samples 0
  done
done
