#!/bin/bash
# Prefill-heavy serving (2048-token prompts, 32 generated): throughput + kernel window.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pf_bench 600 python bench.py --no-operator --batch 256 --prompt-len 2048 --output-len 32 --max-model-len 4096 --steps 60 --warmup 20
step pf_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof99 -o pf -f csv -- python3 bench.py --no-operator --batch 256 --prompt-len 2048 --output-len 32 --max-model-len 4096 --steps 20 --warmup 10
