#!/bin/bash
source scripts/gpu_check.sh
step pytest_attn 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention or attn"
step attn_decode 300 python scripts/bench_decode_attn.py
