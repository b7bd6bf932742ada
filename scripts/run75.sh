#!/bin/bash
# Host-side profile (cProfile) of the default bench: random prompts vs a shared 192-token prefix.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step cprof_random 400 python -m cProfile -o gpurun_out/cprof_random.out bench.py --steps 40 --warmup 5 --no-prefix-cache --no-operator
step cprof_shared 400 python -m cProfile -o gpurun_out/cprof_shared.out bench.py --steps 40 --warmup 5 --no-prefix-cache --no-operator --shared-prefix 192
