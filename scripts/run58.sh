#!/bin/bash
# Per-M GEMV KW=4 default (M <= 2: 8192 sets, else 2048): full GPU suite, smoke, batch 1/2/4/8 decode, default bench.
source scripts/gpu_check.sh
cd "$GRAFT_REPO_ROOT"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 300 python __graft_entry__.py smoke
for b in 1 2 4 8; do
  step b$b 200 python bench.py --batch $b --steps 300 --warmup 20 --no-operator
done
step bench_default 400 python bench.py
