#!/bin/bash
# Tile-order band height (group_m) of the four-wave GEMM at the headline shapes, one process per value.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for g in 1 2 4 8 16; do
  step gm$g 200 env MLOP_GEMM_PP_GROUP_M=$g BENCH_VARIANTS=5 BENCH_MS=4088 python -u scripts/bench_bigm.py
done
