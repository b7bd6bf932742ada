#!/bin/bash
# Batch-1 decode: per-kernel profile + small-M GEMM microbench (before the GEMV kernel).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step prof_b1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b1 -o b --output-format csv -- python3 bench.py --batch 1 --steps 100 --warmup 10 --no-operator
BENCH_MS=1,4,8,16,32,64 step gemm_small 300 python scripts/bench_gemm.py
