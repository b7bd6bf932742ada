#!/bin/bash
# Grouped split-K target (workgroups) 1024 vs 2048 vs 4096 at Mixtral batch 64 / 128.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for t in 1024 2048 4096; do
  step mix_b64_t$t 600 env MLOP_GROUPED_SPLIT_TARGET=$t python bench.py --model mixtral-8x7b --batch 64 --steps 60 --warmup 20 --no-operator
done
step mix_b128_t1024 600 python bench.py --model mixtral-8x7b --batch 128 --steps 60 --warmup 20 --no-operator
step mix_b128_t2048 600 env MLOP_GROUPED_SPLIT_TARGET=2048 python bench.py --model mixtral-8x7b --batch 128 --steps 60 --warmup 20 --no-operator
