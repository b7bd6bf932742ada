#!/bin/bash
# Llama-3-70B batch 256 on one GPU, round-1 flags: hand-written GEMMs (default) vs the
# per-shape table with hipBLASLt (MLOP_GEMM_BACKEND=auto), interleaved
B="python3 bench.py --model llama3-70b --batch 256 --steps 40 --warmup 10 --no-operator --cr-ready-samples 0"
bash scripts/steps.sh "m1 900 $B" "a1 900 env MLOP_GEMM_BACKEND=auto $B" "m2 900 $B"
