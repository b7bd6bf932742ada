#!/bin/bash
# Full GPU tests after today's kernels; mid-batch benches; fresh rocprof of the default bench.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench_b64 300 python bench.py --batch 64 --steps 100 --warmup 20
step bench_b256 300 python bench.py --batch 256 --steps 100 --warmup 20
step prof_default 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_def -o b --output-format csv -- python3 bench.py --steps 60 --warmup 10 --no-operator
