#!/bin/bash
# Ping-pong GEMM diagnostics (DMA latency / DMA issue share) and the fused QKV+RoPE epilogue cost.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step diag_ab 300 env BENCH_DIAG=1 python -u scripts/bench_bigm.py
step qkv_rope 300 env BENCH_MS=2048,4088 MLOP_GEMM_PP_PHASES=2 python -u scripts/bench_qkv_rope.py
