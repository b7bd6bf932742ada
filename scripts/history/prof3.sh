#!/bin/bash
# kernel-time profile of the default bench (Llama-3-8B, B=1024, graphs)
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step bench_plain 600 python bench.py --steps 60 --warmup 30
step prof_bench 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o bench --output-format csv -- python3 bench.py --steps 30 --warmup 20 --no-operator
