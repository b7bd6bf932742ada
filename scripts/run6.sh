#!/bin/bash
source scripts/gpu_check.sh
step pytest_gpu 900 python -m pytest tests -q -m gpu -x
step bench_b256 600 python bench.py --batch 256
step bench_b512 600 python bench.py --batch 512
step bench_b1024 600 python bench.py --batch 1024 --steps 150
