#!/bin/bash
source scripts/gpu_check.sh
step bg_v4 300 env MLOP_GEMM_BIG_VARIANT=4 BENCH_MS=2048,4096 BENCH_TAG=v4 python scripts/bench_gemm.py
step bg_v3 300 env MLOP_GEMM_BIG_VARIANT=3 BENCH_MS=2048,4096 BENCH_TAG=v3 python scripts/bench_gemm.py
