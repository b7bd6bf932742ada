#!/bin/bash
# Lazy-KV tests, then the rest of the GPU suite.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_kv_lazy 300 python -u -m pytest tests/test_kv_lazy_gpu.py -x -v --timeout 120 --timeout-method thread
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
