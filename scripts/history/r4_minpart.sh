#!/bin/bash
# split-KV partition length at small batch: MLOP_ATTN_MIN_PART 128 (default) vs 64 / 32,
# batch 1 and 8, interleaved (fused combine on at every size since 2b446d9)
B="python3 bench.py --steps 100 --warmup 20 --no-operator --cr-ready-samples 0"
bash scripts/steps.sh \
  "p128a 300 $B --batch 1" "p64a 300 env MLOP_ATTN_MIN_PART=64 $B --batch 1" "p32a 300 env MLOP_ATTN_MIN_PART=32 $B --batch 1" \
  "q128 300 $B --batch 8" "q64 300 env MLOP_ATTN_MIN_PART=64 $B --batch 8" "q32 300 env MLOP_ATTN_MIN_PART=32 $B --batch 8" \
  "p128b 300 $B --batch 1" "p64b 300 env MLOP_ATTN_MIN_PART=64 $B --batch 1" "p32b 300 env MLOP_ATTN_MIN_PART=32 $B --batch 1"
