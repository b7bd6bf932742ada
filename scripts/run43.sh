#!/bin/bash
# Concurrency sweep of the headline bench (KV pages sized for the mean context).
source scripts/gpu_check.sh
step bench_c2048 600 python bench.py --steps 100 --warmup 20
step bench_c3072 600 python bench.py --steps 100 --warmup 20 --batch 3072
step bench_c4096 600 python bench.py --steps 100 --warmup 20 --batch 4096 --max-batched-tokens 12288
