#!/bin/bash
# Split top-k/top-p sampling (pre-selection over 16 workgroups per row) at small batch.
source scripts/gpu_check.sh
step pytest_samp 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "sample or argmax"
step b1_sample 300 python bench.py --batch 1 --steps 200 --warmup 20 --no-operator --temperature 0.8
step b8_sample 300 python bench.py --batch 8 --steps 200 --warmup 20 --no-operator --temperature 0.8
step b1_greedy 300 python bench.py --batch 1 --steps 200 --warmup 20 --no-operator
