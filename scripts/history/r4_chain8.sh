#!/bin/bash
# batch 6 / 8 decode: the MFMA small-M path (default, split-K reduce with the add + RMSNorm fused)
# vs the GEMV up to 8 rows with the norm chain (MLOP_GEMV_MAX_M=8 MLOP_GEMV_CHAIN_MAX_M=8) vs the
# GEMV without it; batch 1 once as a regression check of the rebuilt GEMV
B="python3 bench.py --steps 100 --warmup 20 --no-operator --cr-ready-samples 0"
G="env MLOP_GEMV_MAX_M=8 MLOP_GEMV_CHAIN_MAX_M=8"
bash scripts/steps.sh \
  "c8d 300 $B --batch 8" "c8g 300 $G $B --batch 8" "c8n 300 env MLOP_GEMV_MAX_M=8 $B --batch 8" \
  "c6d 300 $B --batch 6" "c6g 300 $G $B --batch 6" \
  "c8d2 300 $B --batch 8" "c8g2 300 $G $B --batch 8" "c1 300 $B --batch 1"
