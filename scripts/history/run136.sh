#!/bin/bash
# Small-M QKV: split-K reduce fused into the RoPE + paged-cache kernel (one launch fewer per
# layer): numerics, then batch 8 / 16 / 32 decode vs the previous build (MLOP_LIB), interleaved.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BASE=$GRAFT_REPO_ROOT/build/ab/_C_base.so
step rope_tests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 150 --timeout-method thread -k "rope or engine or small_tiles"
for r in 1 2; do
  for b in 8 16 32; do
    step e2e_base_${b}_$r 200 env MLOP_LIB=$BASE python bench.py --batch $b --steps 150 --warmup 20 --no-operator
    step e2e_fused_${b}_$r 200 python bench.py --batch $b --steps 150 --warmup 20 --no-operator
  done
done
