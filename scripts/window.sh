#!/bin/bash
# Timed-window kernel profile of one bench configuration: rocprofv3 kernel trace + stats, then
# the per-step breakdown of the last STEPS forwards (trace_window.py).
# Usage: gpurun -- bash scripts/window.sh LABEL STEPS [extra bench.py args...]
#        (env vars before `bash` reach the bench: MLOP_GEMM_BACKEND=auto bash scripts/window.sh ...)
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$1; S=$2; shift 2
step "prof_$L" 600 rocprofv3 --kernel-trace --stats -d "gpurun_out/prof_$L" -o bench --output-format csv -- \
  python3 bench.py --steps "$S" --warmup 10 --no-operator --cr-ready-samples 0 "$@"
step "win_$L" 120 python scripts/trace_window.py "gpurun_out/prof_$L/bench_kernel_trace.csv" --steps "$S" --top 40
rm -f "gpurun_out/prof_$L/bench_kernel_trace.csv"
