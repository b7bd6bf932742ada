#!/bin/bash
# Two-phase ping-pong K-loop: A/B at the headline shapes, then the bench with it (re-tuned
# table; all hand-written).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pp2_ab 300 python -u scripts/bench_bigm.py
step bench_pp2_retune 600 env MLOP_GEMM_PP_PHASES=2 MLOP_GEMM_TABLE=off python -u bench.py --save-gemm-table gpurun_out/gemm_table_pp2.json
step bench_pp2_allmlop 600 env MLOP_GEMM_PP_PHASES=2 MLOP_GEMM_BACKEND=mlop python -u bench.py
