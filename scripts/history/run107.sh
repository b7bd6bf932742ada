#!/bin/bash
# Grouped (MoE) GEMM stream-K A/B at Mixtral sizes (scripts/bench_grouped.py).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step grouped 400 python scripts/bench_grouped.py
