#!/bin/bash
# non-temporal stores (gemm_slab_nt): bit 0 split-K slabs (batch 64 / 256), bit 1 the four-wave
# kernel's C stores (headline); numerics first
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_w4_gpu.py tests/test_norm_chain_gpu.py
for i in 1 2; do
  step "h_off$i" 500 python3 bench.py --no-operator --steps 20 --warmup 5 --cr-ready-samples 0
  step "h_on$i" 500 python3 bench.py --no-operator --steps 20 --warmup 5 --cr-ready-samples 0 --ab-ops gemm_slab_nt=2
done
for i in 1 2; do
  for b in 256 64; do
    step "b${b}_off$i" 300 python3 bench.py --no-operator --batch $b --steps 40 --warmup 10 --cr-ready-samples 0
    step "b${b}_on$i" 300 python3 bench.py --no-operator --batch $b --steps 40 --warmup 10 --cr-ready-samples 0 --ab-ops gemm_slab_nt=1
  done
done
