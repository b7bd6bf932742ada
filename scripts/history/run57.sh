#!/bin/bash
# GEMV KW=4 threshold, second sweep: lm_head into KW=4 (65536) at batch 1; batch 2 / 4 at 2048 vs 8192.
source scripts/gpu_check.sh
cd "$GRAFT_REPO_ROOT"
for t in 8192 65536 8192 65536; do
  MLOP_GEMV_KW4_SETS=$t step b1_kw$t 200 python bench.py --batch 1 --steps 300 --warmup 20 --no-operator
done
for b in 2 4; do for t in 2048 8192 2048 8192; do
  MLOP_GEMV_KW4_SETS=$t step b${b}_kw$t 200 python bench.py --batch $b --steps 300 --warmup 20 --no-operator
done; done
