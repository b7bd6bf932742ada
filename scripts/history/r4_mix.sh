#!/bin/bash
# Mixtral-8x7B on the round-4 tree: batch 1024 window profile, batch 1 and 64 benches
bash scripts/window.sh mix 20 --model mixtral-8x7b --batch 1024 && bash scripts/steps.sh \
  "mix1 600 python3 bench.py --model mixtral-8x7b --batch 1 --steps 100 --warmup 10 --no-operator --cr-ready-samples 0" \
  "mix64 600 python3 bench.py --model mixtral-8x7b --batch 64 --steps 60 --warmup 20 --no-operator --cr-ready-samples 0"
