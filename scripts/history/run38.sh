#!/bin/bash
# K2 GEMV (M <= 8) + split argmax: numerics, GEMV vs old MFMA path vs hipBLASLt, batch-1/8 decode,
# attention partition size sweep at batch 1, refreshed GEMM table, rocprof of batch-1 decode.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_k 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread
BENCH_MS=1,2,4,8 step gemm_new 300 python scripts/bench_gemm.py
MLOP_GEMV_MAX_M=0 BENCH_TAG=old BENCH_MS=1,8 step gemm_old 300 python scripts/bench_gemm.py
step bench_b1 300 python bench.py --batch 1 --steps 200 --warmup 20 --no-operator --save-gemm-table gpurun_out/gemm_table.json
MLOP_ATTN_MIN_PART=128 step bench_b1_p128 300 python bench.py --batch 1 --steps 200 --warmup 20 --no-operator
MLOP_ATTN_MIN_PART=64 step bench_b1_p64 300 python bench.py --batch 1 --steps 200 --warmup 20 --no-operator
step bench_b8 300 python bench.py --batch 8 --steps 200 --warmup 20 --no-operator --save-gemm-table gpurun_out/gemm_table.json
step prof_b1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b1g -o b --output-format csv -- python3 bench.py --batch 1 --steps 100 --warmup 10 --no-operator
