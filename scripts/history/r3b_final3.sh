#!/bin/bash
# Timed-window kernel profile of the last tree (norm chain, S18 / S34 K-loops).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step prof_last 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_last -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 10 --no-operator
step window_last 120 python scripts/trace_window.py gpurun_out/prof_last/bench_kernel_trace.csv --steps 20 --top 30
rm -f gpurun_out/prof_last/bench_kernel_trace.csv
