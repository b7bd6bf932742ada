#!/bin/bash
# Operating-point sweep: concurrency 1536 / 2048 (M ~ 3-4k rows per mixed step) vs 1024.
source scripts/gpu_check.sh
step bench_b2048 600 python bench.py --steps 100 --warmup 40 --batch 2048 --max-model-len 1024
step bench_b1536 600 python bench.py --steps 100 --warmup 40 --batch 1536 --max-model-len 1024
