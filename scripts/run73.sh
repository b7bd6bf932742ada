#!/bin/bash
# HF checkpoints + prefix caching on the GPU engine; default bench (prefix hashing cost on random prompts).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_loader 300 python -u -m pytest tests/test_loader_gpu.py tests/test_model_gpu.py -x -v --timeout 200 --timeout-method thread
step bench_default 400 python bench.py
