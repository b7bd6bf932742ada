#!/bin/bash
# K15 custom all-reduce (2 processes on one GPU via IPC) + the rest of the GPU suite
source scripts/gpu_check.sh
step pytest_car 300 python -m pytest tests/test_custom_ar_gpu.py -q -m gpu -x
step pytest_gpu 900 python -m pytest tests/ -q -m gpu -x
