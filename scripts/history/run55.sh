#!/bin/bash
# Concurrency sweep above the 2048 default (sequences are 512 tokens, so KV for 3072 fits in 288 GB).
source scripts/gpu_check.sh
cd "$GRAFT_REPO_ROOT"
step b3072 400 python bench.py --batch 3072 --steps 100 --warmup 20 --no-operator
step b3072_t12k 400 python bench.py --batch 3072 --max-batched-tokens 12288 --steps 100 --warmup 20 --no-operator
step b2048_t12k 400 python bench.py --batch 2048 --max-batched-tokens 12288 --steps 100 --warmup 20 --no-operator
