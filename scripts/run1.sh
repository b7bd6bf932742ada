#!/bin/bash
source scripts/gpu_check.sh
step pytest_gpu 900 python -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -q -m gpu
step bench_small 600 python bench.py --steps 30 --warmup 10 --no-operator
