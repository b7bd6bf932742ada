#!/bin/bash
# ping-pong GEMM tile-band sweep (group_m m-tiles share a B panel)
source scripts/gpu_check.sh
step pytest_gemm 600 env MLOP_GEMM_PP_GROUP_M=4 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "gemm"
for g in 1 4 8 16; do
  step bg_g$g 300 env BENCH_MS=2048,4096 BENCH_TAG=g$g MLOP_GEMM_PP_GROUP_M=$g python scripts/bench_gemm.py
done
