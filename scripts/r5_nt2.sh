#!/bin/bash
# non-temporal K / V pages in decode attention (attn_kv_nt) on the headline and batch 64, and
# non-temporal expert weights in the grouped ping-pong kernel (gemm_small_nt bit 2) on Mixtral
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  step "h_off$i" 500 python3 bench.py --no-operator --steps 20 --warmup 5 --cr-ready-samples 0
  step "h_on$i" 500 python3 bench.py --no-operator --steps 20 --warmup 5 --cr-ready-samples 0 --ab-ops attn_kv_nt=1
done
for i in 1 2; do
  step "l64_off$i" 300 python3 bench.py --no-operator --batch 64 --steps 60 --warmup 10 --cr-ready-samples 0
  step "l64_on$i" 300 python3 bench.py --no-operator --batch 64 --steps 60 --warmup 10 --cr-ready-samples 0 --ab-ops attn_kv_nt=1
done
for b in 256 1024; do
  for i in 1 2; do
    step "m${b}_off$i" 400 python3 bench.py --no-operator --model mixtral-8x7b --batch $b --steps 30 --warmup 10 --cr-ready-samples 0
    step "m${b}_on$i" 400 python3 bench.py --no-operator --model mixtral-8x7b --batch $b --steps 30 --warmup 10 --cr-ready-samples 0 --ab-ops gemm_small_nt=7
  done
done
