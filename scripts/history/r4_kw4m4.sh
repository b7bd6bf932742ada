#!/bin/bash
# batch 3 / 4 decode: K-split GEMV (KW = 4) below 2048 sets (default) vs below 4096 (o / down /
# QKV then split K over the 4 waves too) vs 8192 (every projection)
B="python3 bench.py --steps 100 --warmup 20 --no-operator --cr-ready-samples 0"
bash scripts/steps.sh \
  "k4d 300 $B --batch 4" "k4a 300 env MLOP_GEMV_KW4_SETS=4096 $B --batch 4" "k4b 300 env MLOP_GEMV_KW4_SETS=8192 $B --batch 4" \
  "k3d 300 $B --batch 3" "k3a 300 env MLOP_GEMV_KW4_SETS=4096 $B --batch 3" \
  "k4d2 300 $B --batch 4" "k4a2 300 env MLOP_GEMV_KW4_SETS=4096 $B --batch 4"
