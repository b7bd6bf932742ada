#!/bin/bash
# Ping-pong GEMM tile-band width (MLOP_GEMM_PP_GROUP_M) at the headline's mixed-step M.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for gm in 1 2 4 8 16; do
  MLOP_GEMM_PP_GROUP_M=$gm BENCH_MS=3840,4096 BENCH_TAG=gm$gm step gemm_gm$gm 200 python scripts/bench_gemm.py
done
