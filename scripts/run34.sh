#!/bin/bash
# Full validation of the restored tree: GPU tests, smoke, default bench.
source scripts/gpu_check.sh
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 600 python bench.py
