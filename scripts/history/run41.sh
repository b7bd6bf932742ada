#!/bin/bash
# Norm fusion at M = 1 only: GPU tests, batch-1 with / without the fused norms (same box), batch 2 / 4.
source scripts/gpu_check.sh
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench_b1 300 python bench.py --batch 1 --steps 300 --warmup 20 --no-operator
MLOP_NORM_FUSION=0 step bench_b1_nofuse 300 python bench.py --batch 1 --steps 300 --warmup 20 --no-operator
step bench_b1_again 300 python bench.py --batch 1 --steps 300 --warmup 20 --no-operator
step bench_b2 300 python bench.py --batch 2 --steps 200 --warmup 20 --no-operator
step bench_b4 300 python bench.py --batch 4 --steps 200 --warmup 20 --no-operator
