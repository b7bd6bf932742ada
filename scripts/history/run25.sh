#!/bin/bash
# Steady-state (ramped) operating-point sweep.
source scripts/gpu_check.sh
step bench_r1024 600 python bench.py --steps 100 --warmup 20 --batch 1024
step bench_r2048 600 python bench.py --steps 100 --warmup 20 --batch 2048 --max-model-len 1024
step bench_r1536 600 python bench.py --steps 100 --warmup 20 --batch 1536 --max-model-len 1024
