#!/bin/bash
# Kernel trace of batch-16 decode with the row-fitted small-M tiles (timed window).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step prof135 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof135 -o b16 --output-format csv -- python3 bench.py --batch 16 --steps 40 --warmup 10 --no-operator
step window135 120 python scripts/trace_window.py gpurun_out/prof135/b16_kernel_trace.csv --steps 30 --top 30
