#!/bin/bash
# batch-1 split-KV partition length: 128 (default) vs 512 / 1024 (one partition: no combine)
B="python3 bench.py --steps 100 --warmup 20 --no-operator --cr-ready-samples 0 --batch 1"
bash scripts/steps.sh \
  "m128a 300 $B" "m512a 300 env MLOP_ATTN_MIN_PART=512 $B" "m1ka 300 env MLOP_ATTN_MIN_PART=1024 $B" \
  "m128b 300 $B" "m512b 300 env MLOP_ATTN_MIN_PART=512 $B" "m1kb 300 env MLOP_ATTN_MIN_PART=1024 $B"
