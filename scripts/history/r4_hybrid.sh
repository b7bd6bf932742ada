#!/bin/bash
# hand-written GEMMs everywhere (default) vs the per-shape timed choice against hipBLASLt below
# 1024 rows (MLOP_GEMM_AUTO_MAX_M=1024), batch 256 / 512 / 768, interleaved
B="python3 bench.py --steps 60 --warmup 10 --no-operator --cr-ready-samples 0"
H="env MLOP_GEMM_AUTO_MAX_M=1024"
bash scripts/steps.sh \
  "y256d 400 $B --batch 256" "y256h 400 $H $B --batch 256" \
  "y512d 400 $B --batch 512" "y512h 400 $H $B --batch 512" \
  "y768d 500 $B --batch 768" "y768h 500 $H $B --batch 768" \
  "y512d2 400 $B --batch 512" "y512h2 400 $H $B --batch 512"
