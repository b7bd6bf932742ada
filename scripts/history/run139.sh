#!/bin/bash
# M 33-64: 6-deep ring on the narrow projections (qkv / o / down) vs the previous build.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BASE=$GRAFT_REPO_ROOT/build/ab/_C_base.so
step m64_tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 150 --timeout-method thread -k "small_tiles or rope_cache_fused"
for r in 1 2; do
  for b in 48 64; do
    step e2e_base_${b}_$r 200 env MLOP_LIB=$BASE python bench.py --batch $b --steps 150 --warmup 20 --no-operator
    step e2e_s6_${b}_$r 200 python bench.py --batch $b --steps 150 --warmup 20 --no-operator
  done
done
