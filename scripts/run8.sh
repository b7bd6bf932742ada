#!/bin/bash
source scripts/gpu_check.sh
step pytest_gemm 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "gemm or moe"
step bg_pipe 300 env BENCH_MS=64,256,512,1024,8192 BENCH_TAG=pipe python scripts/bench_gemm.py
step bg_pipe_split512 300 env BENCH_MS=256,512 BENCH_TAG=split512 MLOP_GEMM_SPLIT_TARGET=512 python scripts/bench_gemm.py
