#!/bin/bash
# Llama-3-8B mid-size batches (64, 256): throughput + kernel window at 64.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step l_b64 600 python bench.py --batch 64 --steps 100 --warmup 20 --no-operator
step l_b256 600 python bench.py --batch 256 --steps 100 --warmup 20 --no-operator
step l_b64_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof111 -o l -f csv -- python3 bench.py --batch 64 --steps 30 --warmup 10 --no-operator
