#!/bin/bash
# gate_up 4-deep ring at M 33-64: in-situ A/B at batch 48 / 64 vs the previous build (3-deep).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BASE=$GRAFT_REPO_ROOT/build/ab/_C_base.so
for r in 1 2; do
  for b in 64 48; do
    step gu_base_${b}_$r 200 env MLOP_LIB=$BASE python bench.py --batch $b --steps 150 --warmup 20 --no-operator
    step gu_s4_${b}_$r 200 python bench.py --batch $b --steps 150 --warmup 20 --no-operator
  done
done
