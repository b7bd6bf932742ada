#!/bin/bash
# Stream-K tail: re-tune the GEMM table with it on, then bench with that table (twice) and
# with stream-K off under the same table.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step bench_tune 600 env MLOP_GEMM_TABLE=off python bench.py --save-gemm-table gpurun_out/gemm_table_r88.json
step bench_sk 600 env MLOP_GEMM_TABLE=gpurun_out/gemm_table_r88.json python bench.py
step bench_nosk 600 env MLOP_GEMM_SK=0 MLOP_GEMM_TABLE=gpurun_out/gemm_table_r88.json python bench.py
step bench_sk2 600 env MLOP_GEMM_TABLE=gpurun_out/gemm_table_r88.json python bench.py
