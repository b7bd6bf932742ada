#!/bin/bash
# Mixtral-8x7B serving throughput at high concurrency (config 5 shape, 1 GPU), + kernel trace.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step mix_b1024 600 python bench.py --model mixtral-8x7b --batch 1024 --steps 60 --warmup 20 --no-operator
step mix_b1024_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof94 -o mix -f csv -- python3 bench.py --model mixtral-8x7b --batch 1024 --steps 20 --warmup 10 --no-operator
