#!/bin/bash
# Mixtral-8x7B mid-size batches (every expert's weights streamed each step): 64 and 256.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step mix_b64 600 python bench.py --model mixtral-8x7b --batch 64 --steps 60 --warmup 20 --no-operator
step mix_b256 600 python bench.py --model mixtral-8x7b --batch 256 --steps 60 --warmup 20 --no-operator
step mix_b64_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof108 -o mix -f csv -- python3 bench.py --model mixtral-8x7b --batch 64 --steps 20 --warmup 10 --no-operator
