#!/bin/bash
# grouped ping-pong nt decided per expert on device (one m-tile = streamed once): Mixtral A/B
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step moe_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "grouped or nt_weight or moe"
for b in 1024 256 512; do
  for i in 1 2; do
    step "m${b}_off$i" 400 python3 bench.py --no-operator --model mixtral-8x7b --batch $b --steps 30 --warmup 10 --cr-ready-samples 0 --ab-ops gemm_small_nt=3
    step "m${b}_on$i" 400 python3 bench.py --no-operator --model mixtral-8x7b --batch $b --steps 30 --warmup 10 --cr-ready-samples 0
  done
done
