#!/bin/bash
# Mixtral-8x7B at concurrency 1024 after the grouped stream-K / flash work: bench + kernel window.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step mix_b1024 600 python bench.py --model mixtral-8x7b --batch 1024 --steps 60 --warmup 20 --no-operator
step mix_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof106 -o mix -f csv -- python3 bench.py --model mixtral-8x7b --batch 1024 --steps 20 --warmup 10 --no-operator
