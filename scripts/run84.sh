#!/bin/bash
# GEMM autotune keys every 256 rows above M=256 (vs power-of-two buckets), same box:
# old keys + shipped table, then new keys timed from scratch (table off, saved), then new keys + that table.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step bench_pow2 600 env MLOP_GEMM_MBUCKET=pow2 python bench.py
step bench_new_tune 600 env MLOP_GEMM_TABLE=off python bench.py --save-gemm-table gpurun_out/gemm_table_r84.json
step bench_new_table 600 env MLOP_GEMM_TABLE=gpurun_out/gemm_table_r84.json python bench.py
