#!/bin/bash
# Host-side (Python) profile of the default bench: where the ~2 ms per-step gap goes.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step hostprof 600 python -u -m cProfile -o gpurun_out/bench_host.prof bench.py --steps 30 --warmup 5 --no-operator
