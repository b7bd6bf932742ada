#!/bin/bash
# Decode-size GEMMs (M = 32 / 64 / 128): split-K target / tile threshold sweep (bench_proj).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export BENCH_MS=32,64,128
step p_default 200 python scripts/bench_proj.py
step p_t512 200 env MLOP_GEMM_SPLIT_TARGET=512 python scripts/bench_proj.py
step p_t1024 200 env MLOP_GEMM_SPLIT_TARGET=1024 python scripts/bench_proj.py
step p_t1024_m512 200 env MLOP_GEMM_SPLIT_TARGET=1024 MLOP_GEMM_SPLIT_MAX_TILES=512 python scripts/bench_proj.py
