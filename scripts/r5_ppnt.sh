#!/bin/bash
# non-temporal C stores of the ping-pong kernel (gemm_slab_nt bit 2): Mixtral 256 / 1024, Llama 512
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "grouped or gemm or nt_"
for i in 1 2; do
  for b in 1024 256; do
    step "m${b}_off$i" 400 python3 bench.py --no-operator --model mixtral-8x7b --batch $b --steps 30 --warmup 10 --cr-ready-samples 0
    step "m${b}_on$i" 400 python3 bench.py --no-operator --model mixtral-8x7b --batch $b --steps 30 --warmup 10 --cr-ready-samples 0 --ab-ops gemm_slab_nt=7
  done
  step "l512_off$i" 300 python3 bench.py --no-operator --batch 512 --steps 40 --warmup 10 --cr-ready-samples 0
  step "l512_on$i" 300 python3 bench.py --no-operator --batch 512 --steps 40 --warmup 10 --cr-ready-samples 0 --ab-ops gemm_slab_nt=7
done
