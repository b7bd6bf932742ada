#!/bin/bash
# final-tree batch sweep (Llama-3-8B engine-direct) + other families, one box
source scripts/gpu_check.sh
for b in 1 4 16 64 256 512 1024 2048; do
  step "sw_b$b" 300 python3 bench.py --no-operator --batch $b --steps 40 --warmup 10 --cr-ready-samples 0
done
step sw_mix1 300 python3 bench.py --no-operator --model mixtral-8x7b --batch 1 --steps 40 --warmup 10 --cr-ready-samples 0
step sw_mix64 300 python3 bench.py --no-operator --model mixtral-8x7b --batch 64 --steps 30 --warmup 10 --cr-ready-samples 0
step sw_70b1 400 python3 bench.py --no-operator --model llama3-70b --batch 1 --steps 30 --warmup 5 --cr-ready-samples 0
step sw_driver 400 python3 bench.py --gpus 1 --steps 20 --warmup 5
