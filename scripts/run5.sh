#!/bin/bash
source scripts/gpu_check.sh
step pytest_gemm 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "gemm or moe"
step bg_default 300 env BENCH_MS=64,256,512,8192 BENCH_TAG=default python scripts/bench_gemm.py
step bg_split512 300 env BENCH_MS=256,512 BENCH_TAG=split512 MLOP_GEMM_SPLIT_TARGET=512 python scripts/bench_gemm.py
step bg_bn128 300 env BENCH_MS=256,512 BENCH_TAG=bn128 MLOP_GEMM_BN128_MIN_TILES=1 python scripts/bench_gemm.py
