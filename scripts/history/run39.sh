#!/bin/bash
# GEMV at M <= 4 + cold-cache autotune: kernel tests, batch 1/2/4 decode (table refresh), default bench.
source scripts/gpu_check.sh
step pytest_k 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread
step bench_b1 300 python bench.py --batch 1 --steps 200 --warmup 20 --no-operator --save-gemm-table gpurun_out/gemm_table.json
MLOP_ATTN_MIN_PART=128 step bench_b1_p128 300 python bench.py --batch 1 --steps 200 --warmup 20 --no-operator
MLOP_ATTN_MIN_PART=512 step bench_b1_p512 300 python bench.py --batch 1 --steps 200 --warmup 20 --no-operator
step bench_b2 300 python bench.py --batch 2 --steps 200 --warmup 20 --no-operator --save-gemm-table gpurun_out/gemm_table.json
step bench_b4 300 python bench.py --batch 4 --steps 200 --warmup 20 --no-operator --save-gemm-table gpurun_out/gemm_table.json
step bench_b8 300 python bench.py --batch 8 --steps 200 --warmup 20 --no-operator --save-gemm-table gpurun_out/gemm_table.json
step bench_default 600 python bench.py
