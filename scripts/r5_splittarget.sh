#!/bin/bash
# small-M split-K target 256 vs 512 workgroups (gemm_split_target) at batch 16 / 64 / 256
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  for b in 16 64 256; do
    step "b${b}_t256_$i" 300 python3 bench.py --no-operator --batch $b --steps 60 --warmup 10 --cr-ready-samples 0
    step "b${b}_t512_$i" 300 python3 bench.py --no-operator --batch $b --steps 60 --warmup 10 --cr-ready-samples 0 --ab-ops gemm_split_target=512
  done
done
