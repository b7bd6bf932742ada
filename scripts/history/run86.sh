#!/bin/bash
# Robust autotune (best of 3 interleaved rounds x 5 calls) with 256-row keys: re-tune from
# scratch and save the table, then bench with it; the shipped table + pow2 keys for reference.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step bench_tune 600 env MLOP_GEMM_TABLE=off python bench.py --save-gemm-table gpurun_out/gemm_table_r86.json
step bench_table 600 env MLOP_GEMM_TABLE=gpurun_out/gemm_table_r86.json python bench.py
step bench_pow2 600 env MLOP_GEMM_MBUCKET=pow2 python bench.py
step bench_table2 600 env MLOP_GEMM_TABLE=gpurun_out/gemm_table_r86.json python bench.py
