#!/bin/bash
# narrow mid-M GEMMs on the 256x128 kernel: split-K target (MLOP_GEMM_SPLIT_TARGET, default 256) 512 / 1024
G="python3 scripts/bench_gemm.py"
bash scripts/steps.sh \
  "ms_d 600 env BENCH_MS=512,768,1024 BENCH_TAG=d $G" \
  "ms_512 600 env BENCH_MS=512,768,1024 MLOP_GEMM_SPLIT_TARGET=512 BENCH_TAG=s512 $G" \
  "ms_1k 600 env BENCH_MS=512,768,1024 MLOP_GEMM_SPLIT_TARGET=1024 BENCH_TAG=s1k $G"
