#!/bin/bash
# rocprofv3 kernel profile of batch-1 decode with the per-M GEMV KW=4 default.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step prof_b1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b1 -o b1 --output-format csv -- python3 bench.py --batch 1 --steps 100 --warmup 10 --no-operator
find gpurun_out/prof_b1 -name "*kernel_stats.csv" -exec cp {} gpurun_out/b1_kernel_stats.csv \;
