#!/bin/bash
# Hand-written GEMM vs hipBLASLt at the headline's step sizes (M = 2048 decode-only, ~3840 mixed).
source scripts/gpu_check.sh
BENCH_MS=2048,3840,4096 step gemm_big 300 python scripts/bench_gemm.py
