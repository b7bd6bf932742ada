#!/bin/bash
# start-up breakdown (model build / KV alloc / graph capture) on two back-to-back benches
source scripts/gpu_check.sh
step b_first 600 python bench.py --steps 100 --warmup 40
step b_second 600 python bench.py --steps 100 --warmup 40
