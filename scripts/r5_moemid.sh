#!/bin/bash
# mid-size MoE dispatch (one launch, experts read x through arow): numerics, then Mixtral serving
source scripts/gpu_check.sh
step moe_tests 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "moe or mixtral or grouped"
step mix64 300 python3 bench.py --no-operator --model mixtral-8x7b --batch 64 --steps 30 --warmup 10 --cr-ready-samples 0
step mix32 300 python3 bench.py --no-operator --model mixtral-8x7b --batch 32 --steps 30 --warmup 10 --cr-ready-samples 0
step mix256 300 python3 bench.py --no-operator --model mixtral-8x7b --batch 256 --steps 30 --warmup 10 --cr-ready-samples 0
bash scripts/window.sh mix64b 20 --model mixtral-8x7b --batch 64
