#!/bin/bash
# Mixed-step token budget sweep: M per step vs the 256x256 tile waves (16 m-tiles = 4096 rows).
source scripts/gpu_check.sh
step bench_t8192 600 python bench.py --steps 100 --warmup 20
step bench_t4096 600 python bench.py --steps 100 --warmup 20 --max-batched-tokens 4096
step bench_t4352 600 python bench.py --steps 100 --warmup 20 --max-batched-tokens 4352
step bench_t4608 600 python bench.py --steps 100 --warmup 20 --max-batched-tokens 4608
