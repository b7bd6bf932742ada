#!/bin/bash
# GEMM at the mixed-step M range (decode batch + prompt chunk): ours (v0 / v1) vs hipBLASLt
source scripts/gpu_check.sh
step pytest_k 600 python -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -q -m gpu -x -k "argmax or engine or llama3"
step bg_v0 400 env BENCH_MS=1536,2048,3072,4096 BENCH_TAG=v0 python scripts/bench_gemm.py
step bg_v1 400 env BENCH_MS=1536,2048,3072,4096 BENCH_TAG=v1 MLOP_GEMM_BIG_VARIANT=1 MLOP_GEMM_BIG_MIN_M=1024 python scripts/bench_gemm.py
step bench_attn 300 python scripts/bench_attn.py
