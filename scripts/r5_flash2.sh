#!/bin/bash
# K7 flash prefill variants: numerics, then the microbench at 3 shapes
source scripts/gpu_check.sh
step flash_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash or paged_attention"
step flash_8192 200 env S=1 L=8192 python -u scripts/bench_flash.py
step flash_2048 200 env S=4 L=2048 python -u scripts/bench_flash.py
step flash_512 200 env S=16 L=512 python -u scripts/bench_flash.py
step flash_32k 200 env S=1 L=32768 ITERS=5 python -u scripts/bench_flash.py
