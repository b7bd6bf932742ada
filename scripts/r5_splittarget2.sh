#!/bin/bash
# split-K target of the <= 32-row tiles (gemm_split_target, default 512) vs 256 at batch 32 / 24 / 16
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or rope or norm"
for i in 1 2; do
  for b in 32 24 16; do
    step "b${b}_t256_$i" 300 python3 bench.py --no-operator --batch $b --steps 60 --warmup 10 --cr-ready-samples 0 --ab-ops gemm_split_target=256
    step "b${b}_t512_$i" 300 python3 bench.py --no-operator --batch $b --steps 60 --warmup 10 --cr-ready-samples 0
  done
done
