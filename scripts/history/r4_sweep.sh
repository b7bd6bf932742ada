#!/bin/bash
# batch sweep on the round-4 final tree (Llama-3-8B, 256 + 256 tokens, engine-direct)
B="python3 bench.py --no-operator --cr-ready-samples 0"
bash scripts/steps.sh \
  "s1 300 $B --batch 1 --steps 100 --warmup 20" "s4 300 $B --batch 4 --steps 100 --warmup 20" \
  "s16 300 $B --batch 16 --steps 100 --warmup 20" "s64 300 $B --batch 64 --steps 100 --warmup 20" \
  "s256 400 $B --batch 256 --steps 60 --warmup 10" "s512 400 $B --batch 512 --steps 60 --warmup 10" \
  "s1024 500 $B --batch 1024 --steps 60 --warmup 10" "s2048 600 $B --batch 2048 --steps 20 --warmup 5"
