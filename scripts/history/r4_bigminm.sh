#!/bin/bash
# mid-M GEMMs (M 256-1024): the large-M kernels (four-wave / ping-pong) from MLOP_GEMM_BIG_MIN_M
# rows (default 1024) vs 512 / 256, Llama-3-8B and -70B shapes, hand-written vs hipBLASLt
G="python3 scripts/bench_gemm.py"
bash scripts/steps.sh \
  "bm_d 600 env BENCH_MS=256,512,1024 BENCH_TAG=d $G" \
  "bm_512 600 env BENCH_MS=512,1024 MLOP_GEMM_BIG_MIN_M=512 BENCH_TAG=m512 $G" \
  "bm_256 600 env BENCH_MS=256,512 MLOP_GEMM_BIG_MIN_M=256 BENCH_TAG=m256 $G" \
  "bm70_256 600 env BENCH_MODEL=70b BENCH_MS=256,512 MLOP_GEMM_BIG_MIN_M=256 BENCH_TAG=m256_70b $G"
