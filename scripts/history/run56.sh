#!/bin/bash
# GEMV KW=4 threshold (waves of a workgroup split K) at batch-1 decode: 2048 (default) vs 4096 vs 8192 sets.
source scripts/gpu_check.sh
cd "$GRAFT_REPO_ROOT"
export MLOP_GEMV_KW4_SETS=8192
step gemv_tests_kw8192 300 python -u -m pytest tests -m gpu -x -q -k "gemv or Gemv or decode" --timeout 120 --timeout-method thread
unset MLOP_GEMV_KW4_SETS
for t in 2048 4096 8192 2048 4096 8192; do
  MLOP_GEMV_KW4_SETS=$t step b1_kw$t 200 python bench.py --batch 1 --steps 300 --warmup 20 --no-operator
done
