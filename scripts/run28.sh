#!/bin/bash
source scripts/gpu_check.sh
step pytest_rope 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "rope"
step bench_qkv_rope 300 python scripts/bench_qkv_rope.py
