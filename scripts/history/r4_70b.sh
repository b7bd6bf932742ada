#!/bin/bash
# Llama-3-70B bf16 on one GPU, batch 1: the GEMV norm chain (default) vs MLOP_GEMV_CHAIN=0
B="python3 bench.py --model llama3-70b --batch 1 --steps 40 --warmup 10 --no-operator --cr-ready-samples 0"
bash scripts/steps.sh "l70c 600 $B" "l70n 600 env MLOP_GEMV_CHAIN=0 $B"
