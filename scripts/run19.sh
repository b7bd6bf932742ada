#!/bin/bash
# ping-pong 256x256 GEMM: numerics, then the mixed-step M range vs hipBLASLt
source scripts/gpu_check.sh
step pytest_gemm 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "gemm or moe"
step bg_pp 400 env BENCH_MS=1024,2048,4096,8192 BENCH_TAG=pp python scripts/bench_gemm.py
