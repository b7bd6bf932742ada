#!/bin/bash
# Kernel trace of the current default bench's timed window (refresh of r02_bench_default_window).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step prof128 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof128 -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 10 --no-operator
step window128 120 python scripts/trace_window.py gpurun_out/prof128/bench_kernel_trace.csv --steps 20 --top 40
rm -f gpurun_out/prof128/bench_kernel_trace.csv.gz
