#!/bin/bash
# Default bench (driver invocation), then the timed-window kernel profile.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step bench 600 python -u bench.py
step bench_sync 600 python -u bench.py --no-async
step prof_w4b 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_w4b -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 10 --no-operator
step window_w4b 120 python scripts/trace_window.py gpurun_out/prof_w4b/bench_kernel_trace.csv --steps 20 --top 40
rm -f gpurun_out/prof_w4b/bench_kernel_trace.csv.gz
