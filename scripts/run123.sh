#!/bin/bash
# K7 flash prefill unrolled by the LDS ring depth (slot offsets as ds_read immediates):
# numerics, then in-process A/B against the previous build (MLOP_LIB), alternating; then the
# default bench saving the GEMM table over the new 10k-row step range.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BASE=$GRAFT_REPO_ROOT/build/ab/_C_base.so
step kern 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread -k "attention or flash or engine or prefix"
for r in 1 2; do
  for sl in "4 2048" "1 8192" "16 512"; do
    set -- $sl
    step fu_base_${1}x${2}_$r 120 env MLOP_LIB=$BASE S=$1 L=$2 python scripts/bench_flash.py
    step fu_new_${1}x${2}_$r 120 env S=$1 L=$2 python scripts/bench_flash.py
  done
done
step bench_table 400 python bench.py --save-gemm-table gpurun_out/gemm_table_new.json
