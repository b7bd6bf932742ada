#!/bin/bash
source scripts/gpu_check.sh
step pytest_gemm 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "gemm or moe"
step pytest_gemm_v1 600 env MLOP_GEMM_BIG_VARIANT=1 MLOP_GEMM_BIG_MIN_M=257 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "gemm"
step bg_v0 300 env BENCH_MS=64,256,1024,8192 BENCH_TAG=v0 python scripts/bench_gemm.py
step bg_v1 300 env BENCH_MS=1024,8192 BENCH_TAG=v1 MLOP_GEMM_BIG_VARIANT=1 python scripts/bench_gemm.py
