#!/bin/bash
# Row-scaled variants on the S18 / S34 K-loops (the two row-sum DMAs counted in the first wait):
# numerics (multi-tile gate_up exercises the count), microbench, same-box A/B.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step t_chain6 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_norm_chain_gpu.py tests/test_gemm_w4_gpu.py
step bench_chain6 300 python -u scripts/bench_chain.py
B="python3 bench.py --gpus 1 --steps 100 --warmup 10"
for i in 1 2; do
  step ab6_on_$i 400 $B
  step ab6_off_$i 400 env MLOP_NORM_CHAIN=0 $B
done
