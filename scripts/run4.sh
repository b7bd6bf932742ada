#!/bin/bash
source scripts/gpu_check.sh
step pytest_gpu 900 python -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -q -m gpu -x
step bench_gemm 600 python scripts/bench_gemm.py
step bench 900 python bench.py
