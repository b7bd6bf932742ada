#!/bin/bash
# Prefix cache: host cost on random prompts (default bench, cache on / off), and the gain with a
# 192-token shared system prompt; batch-1 decode.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step bench_default 400 python bench.py
step bench_nocache 400 python bench.py --no-prefix-cache
step bench_shared192 400 python bench.py --shared-prefix 192
step bench_shared192_nocache 400 python bench.py --shared-prefix 192 --no-prefix-cache
step b1 300 python bench.py --batch 1 --steps 300 --warmup 20 --no-operator
