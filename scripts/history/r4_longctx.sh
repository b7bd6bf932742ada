#!/bin/bash
# long-context runs on the current tree (split-KV partitions combined in-launch at every size)
B="python3 bench.py --no-operator --cr-ready-samples 0"
bash scripts/steps.sh \
  "lc32k 900 $B --model llama3.1-8b --batch 16 --prompt-len 32000 --output-len 256 --max-model-len 32768 --steps 100 --warmup 10" \
  "lc32kr 900 env MLOP_ATTN_FUSED_MAX_PAIRS=32 $B --model llama3.1-8b --batch 16 --prompt-len 32000 --output-len 256 --max-model-len 32768 --steps 100 --warmup 10"
