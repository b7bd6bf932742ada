#!/bin/bash
# Re-validation after the container rebuild: GPU suite, smoke, default bench (driver's invocation).
source scripts/gpu_check.sh
cd "$GRAFT_REPO_ROOT"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 300 python __graft_entry__.py smoke
step bench_default 400 python bench.py
step b1 300 python bench.py --batch 1 --steps 200 --warmup 20 --no-operator
