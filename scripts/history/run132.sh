#!/bin/bash
# Row-fitted small-M tiles ON by default + re-tuned small-M table entries vs the previous default
# (64 x 64 tiles, previous table), end to end at batch 8 / 16 / 32, interleaved.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for b in 8 16 32; do
    step e2e_old_${b}_$r 200 env MLOP_GEMM_SMALL_TILE=0 MLOP_GEMM_TABLE=build/tables/old.json python bench.py --batch $b --steps 150 --warmup 20 --no-operator
    step e2e_new_${b}_$r 200 python bench.py --batch $b --steps 150 --warmup 20 --no-operator
  done
done
