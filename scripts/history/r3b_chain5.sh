#!/bin/bash
# ADD epilogue with the next row block's residual loads issued early: numerics, microbench, A/B.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step t_chain5 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_norm_chain_gpu.py
step bench_chain5 300 python -u scripts/bench_chain.py
B="python3 bench.py --gpus 1 --steps 100 --warmup 10"
for i in 1 2; do
  step ab5_on_$i 400 $B
  step ab5_off_$i 400 env MLOP_NORM_CHAIN=0 $B
done
