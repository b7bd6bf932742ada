#!/bin/bash
# Kernel trace of the default bench's timed window (hand-written GEMMs by default).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step prof_r3 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3 -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 10 --no-operator
step window_r3 120 python scripts/trace_window.py gpurun_out/prof_r3/bench_kernel_trace.csv --steps 20 --top 40
rm -f gpurun_out/prof_r3/bench_kernel_trace.csv.gz
