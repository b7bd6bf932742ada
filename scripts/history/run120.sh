#!/bin/bash
# Long context end to end (SURVEY §5 "long-context"): Llama-3.1-8B (llama3 RoPE scaling,
# 128k positions) and Mixtral-8x7B (32k) with 32k / 100k-token prompts served through chunked
# prefill (8k-token chunks) + paged KV + split-KV decode partitions.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step lc_l31_32k 400 python bench.py --no-operator --model llama3.1-8b --batch 16 --prompt-len 32000 --output-len 256 --max-model-len 32768 --steps 100 --warmup 10
step lc_l31_100k 400 python bench.py --no-operator --model llama3.1-8b --batch 4 --prompt-len 100000 --output-len 256 --max-model-len 131072 --steps 100 --warmup 10
step lc_mixtral30k 500 python bench.py --no-operator --model mixtral-8x7b --batch 4 --prompt-len 30000 --output-len 256 --max-model-len 32768 --steps 60 --warmup 10
