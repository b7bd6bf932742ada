#!/bin/bash
# Llama-3-70B batch-1 decode (TP=1, 141 GB): per-M GEMV KW=4 default vs the old 2048-set threshold.
source scripts/gpu_check.sh
cd "$GRAFT_REPO_ROOT"
step b1_70b_default 300 python bench.py --model llama3-70b --batch 1 --steps 60 --warmup 10 --no-operator
MLOP_GEMV_KW4_SETS=2048 step b1_70b_kw2048 300 python bench.py --model llama3-70b --batch 1 --steps 60 --warmup 10 --no-operator
step b1_mixtral_default 300 python bench.py --model mixtral-8x7b --batch 1 --steps 100 --warmup 10 --no-operator
MLOP_GEMV_KW4_SETS=2048 step b1_mixtral_kw2048 300 python bench.py --model mixtral-8x7b --batch 1 --steps 100 --warmup 10 --no-operator
