#!/bin/bash
source scripts/gpu_check.sh
export BENCH_MS=64,256,8192
BENCH_TAG=default step bg_default 300 python scripts/bench_gemm.py
BENCH_TAG=split512 MLOP_GEMM_SPLIT_TARGET=512 step bg_split512 300 python scripts/bench_gemm.py
BENCH_TAG=split256 MLOP_GEMM_SPLIT_TARGET=256 step bg_split256 300 python scripts/bench_gemm.py
BENCH_TAG=bn128 MLOP_GEMM_BN128_MIN_TILES=1 step bg_bn128 300 python scripts/bench_gemm.py
