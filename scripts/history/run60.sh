#!/bin/bash
# Norm-prologue fusion (MLOP_NORM_FUSION=1) re-measured now that gate_up runs K-split (KW=4) at M <= 2.
source scripts/gpu_check.sh
cd "$GRAFT_REPO_ROOT"
MLOP_NORM_FUSION=1 step norm_tests 300 python -u -m pytest tests -m gpu -x -q -k "norm or engine or decode" --timeout 120 --timeout-method thread
for f in 0 1 0 1; do
  MLOP_NORM_FUSION=$f step b1_nf$f 200 python bench.py --batch 1 --steps 300 --warmup 20 --no-operator
done
for f in 0 1; do
  MLOP_NORM_FUSION=$f step b2_nf$f 200 python bench.py --batch 2 --steps 300 --warmup 20 --no-operator
done
