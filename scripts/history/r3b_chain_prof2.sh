#!/bin/bash
# Same-box timed-window kernel profiles, norm chain on and off.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P="python3 bench.py --steps 40 --warmup 10 --no-operator"
step prof_on 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_on -o bench --output-format csv -- $P
step win_on 120 python scripts/trace_window.py gpurun_out/prof_on/bench_kernel_trace.csv --steps 40 --top 30
rm -f gpurun_out/prof_on/bench_kernel_trace.csv
export MLOP_NORM_CHAIN=0
step prof_off 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_off -o bench --output-format csv -- $P
step win_off 120 python scripts/trace_window.py gpurun_out/prof_off/bench_kernel_trace.csv --steps 40 --top 30
rm -f gpurun_out/prof_off/bench_kernel_trace.csv
