#!/bin/bash
# Timed-window kernel profile with the norm chain on (compare profiles/r03_bench_window_final.md).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step prof_chain 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_chain -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 10 --no-operator
step window_chain 120 python scripts/trace_window.py gpurun_out/prof_chain/bench_kernel_trace.csv --steps 20 --top 40
rm -f gpurun_out/prof_chain/bench_kernel_trace.csv
