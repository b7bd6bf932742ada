#!/bin/bash
# Llama-3-70B bf16 on ONE GPU (141 GB of weights in 288 GB HBM) at batch 256 and 1024: the
# config-4 model's shapes through the hand-written GEMMs / attention at serving batch sizes
B="python3 bench.py --model llama3-70b --steps 20 --warmup 5 --no-operator --cr-ready-samples 0"
bash scripts/steps.sh "l70b256 900 $B --batch 256" "l70b1k 900 $B --batch 1024 --kv-gb 100"
