#!/bin/bash
# Kernel breakdown of the new default operating point (2048 concurrent) + a 3072 probe.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step prof_b2048 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b2048 -o bench --output-format csv -- python3 bench.py --steps 60 --warmup 10 --no-operator
step bench_b3072 600 python bench.py --steps 60 --warmup 10 --batch 3072
