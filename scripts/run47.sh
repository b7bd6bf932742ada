#!/bin/bash
# Sampling cost at small batch (temperature 0.8, top-k 50) vs greedy.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step b1_greedy 300 python bench.py --batch 1 --steps 200 --warmup 20 --no-operator
step b1_sample 300 python bench.py --batch 1 --steps 200 --warmup 20 --no-operator --temperature 0.8
step b8_sample 300 python bench.py --batch 8 --steps 200 --warmup 20 --no-operator --temperature 0.8
step prof_sample 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_samp -o b --output-format csv -- python3 bench.py --batch 1 --steps 100 --warmup 10 --no-operator --temperature 0.8
