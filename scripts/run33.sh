#!/bin/bash
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step prof_mixtral 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mixtral -o b --output-format csv -- python3 bench.py --model mixtral-8x7b --batch 512 --steps 40 --warmup 5 --no-operator
step prof_70b 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_70b -o b --output-format csv -- python3 bench.py --model llama3-70b --batch 256 --steps 30 --warmup 5 --no-operator
