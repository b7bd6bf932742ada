#!/bin/bash
# Grouped (MoE) decode GEMV: kernel + model tests, Mixtral batch 1 / 4 / 512.
source scripts/gpu_check.sh
step pytest_k 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread
step mixtral_b1 300 python bench.py --model mixtral-8x7b --batch 1 --steps 100 --warmup 10 --no-operator
step mixtral_b4 300 python bench.py --model mixtral-8x7b --batch 4 --steps 100 --warmup 10 --no-operator
step mixtral_b512 400 python bench.py --model mixtral-8x7b --batch 512 --steps 60 --warmup 10 --no-operator
