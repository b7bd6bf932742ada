#!/bin/bash
# K7 final kernel: attention numerics + model tests through it, microbench, and a long-prompt serving run
source scripts/gpu_check.sh
step flash_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "flash or paged_attention or prefill or model"
step flash_8192 200 env S=1 L=8192 python -u scripts/bench_flash.py
step flash_2048 200 env S=4 L=2048 python -u scripts/bench_flash.py
step longprompt 400 python3 bench.py --no-operator --batch 256 --prompt-len 2048 --output-len 32 --max-model-len 2304 --steps 20 --warmup 5 --cr-ready-samples 0
