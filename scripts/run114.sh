#!/bin/bash
# Re-validation after the container was re-created (session 3 of round 2):
# GPU suite, smoke, default bench.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 300 python __graft_entry__.py smoke
step bench_default 400 python bench.py
