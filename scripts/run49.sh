#!/bin/bash
# Split-K target sweep of the MFMA path at mid decode sizes (M = 8 .. 64).
source scripts/gpu_check.sh
for t in 320 256 512 768 1024; do
  MLOP_GEMM_SPLIT_TARGET=$t BENCH_TAG=split$t BENCH_MS=8,16,32,64 step gemm_split$t 200 python scripts/bench_gemm.py
done
