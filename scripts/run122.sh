#!/bin/bash
# DPP / permlane-swap cross-lane reductions (no ds_bpermute) + attention built without NaN
# canonicalisation: numerics, then in-process A/B against the previous build (MLOP_LIB) on one box:
# flash prefill microbench and batch-1 decode, alternating.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BASE=$GRAFT_REPO_ROOT/build/ab/_C_base.so
step kern 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_races_gpu.py -x -q --timeout 200 --timeout-method thread -k "attention or flash or gemv or rmsnorm or moe or race or contention or argmax or sample"
for r in 1 2; do
  for sl in "4 2048" "1 8192" "16 512"; do
    set -- $sl
    step fl_base_${1}x${2}_$r 120 env MLOP_LIB=$BASE S=$1 L=$2 python scripts/bench_flash.py
    step fl_new_${1}x${2}_$r 120 env S=$1 L=$2 python scripts/bench_flash.py
  done
  step b1_base_$r 300 env MLOP_LIB=$BASE python bench.py --batch 1 --steps 300 --warmup 20 --no-operator
  step b1_new_$r 300 python bench.py --batch 1 --steps 300 --warmup 20 --no-operator
done
