#!/bin/bash
# Mixtral-8x7B batch-1 decode kernel breakdown after the one-launch MoE dispatch.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step prof_mixtral_b1 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof79 -o mix -f csv -- python3 bench.py --model mixtral-8x7b --batch 1 --steps 50 --warmup 10 --no-operator
