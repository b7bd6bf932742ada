#!/bin/bash
# decode attention's split-KV target grid (MLOP_ATTN_TARGET_WGS, default 1024) at batch 16 / 64
B="python3 bench.py --steps 100 --warmup 20 --no-operator --cr-ready-samples 0"
bash scripts/steps.sh \
  "w1k64 300 $B --batch 64" "w2k64 300 env MLOP_ATTN_TARGET_WGS=2048 $B --batch 64" "w4k64 300 env MLOP_ATTN_TARGET_WGS=4096 $B --batch 64" \
  "w1k16 300 $B --batch 16" "w2k16 300 env MLOP_ATTN_TARGET_WGS=2048 $B --batch 16" "w4k16 300 env MLOP_ATTN_TARGET_WGS=4096 $B --batch 16" \
  "w1k64b 300 $B --batch 64" "w2k64b 300 env MLOP_ATTN_TARGET_WGS=2048 $B --batch 64" "w4k64b 300 env MLOP_ATTN_TARGET_WGS=4096 $B --batch 64"
