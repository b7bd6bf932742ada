#!/bin/bash
# mid-M GEMMs: M = 768 / 1024 / 1536 on the older 256x128 kernel (MLOP_GEMM_BIG_MIN_M=4096) vs
# the default (large-M kernels from 1024 rows), 8B and 70B shapes
G="python3 scripts/bench_gemm.py"
bash scripts/steps.sh \
  "b2_d 600 env BENCH_MS=768,1024,1536 BENCH_TAG=d $G" \
  "b2_v0 600 env BENCH_MS=768,1024,1536 MLOP_GEMM_BIG_MIN_M=4096 BENCH_TAG=v0 $G" \
  "b2_512 600 env BENCH_MS=768 MLOP_GEMM_BIG_MIN_M=512 BENCH_TAG=m512 $G" \
  "b270_d 600 env BENCH_MODEL=70b BENCH_MS=1024 BENCH_TAG=d70 $G" \
  "b270_v0 600 env BENCH_MODEL=70b BENCH_MS=1024 MLOP_GEMM_BIG_MIN_M=4096 BENCH_TAG=v0_70 $G"
