#!/bin/bash
# batch 512 / 1024 serving: hand-written GEMMs (default) vs the per-shape table with hipBLASLt
B="python3 bench.py --steps 60 --warmup 10 --no-operator --cr-ready-samples 0"
bash scripts/steps.sh \
  "am512 600 $B --batch 512" "aa512 600 env MLOP_GEMM_BACKEND=auto $B --batch 512" \
  "am1k 600 $B --batch 1024" "aa1k 600 env MLOP_GEMM_BACKEND=auto $B --batch 1024"
