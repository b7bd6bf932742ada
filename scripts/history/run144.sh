#!/bin/bash
# Kernel trace of batch-64 decode after the small-M tile work (timed window).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step prof144 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof144 -o b64 --output-format csv -- python3 bench.py --batch 64 --steps 40 --warmup 10 --no-operator
step window144 120 python scripts/trace_window.py gpurun_out/prof144/b64_kernel_trace.csv --steps 30 --top 24
