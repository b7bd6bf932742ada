#!/bin/bash
# Round-2 re-validation after container re-creation: GPU suite, smoke, default bench, kernel profile.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 300 python __graft_entry__.py smoke
step bench_default 400 python bench.py
step prof_bench 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof62 -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 10 --no-operator
