#!/bin/bash
source scripts/gpu_check.sh
step pytest_gemm 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "gemm"
step bg_pp2 400 env BENCH_MS=1024,2048,4096,8192 BENCH_TAG=pp2 python scripts/bench_gemm.py
