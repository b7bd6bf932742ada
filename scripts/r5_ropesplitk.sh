#!/bin/bash
# small-M QKV + RoPE with K split (gemm_rope_split 1 / 2 / 4) at batch 16 and 12: numerics, A/B
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "rope or qkv or model"
for i in 1 2; do
  for b in 16 12; do
    for s in 1 2 4; do
      step "b${b}_k${s}_$i" 300 python3 bench.py --no-operator --batch $b --steps 60 --warmup 10 --cr-ready-samples 0 --ab-ops gemm_rope_split=$s
    done
  done
done
