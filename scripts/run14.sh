#!/bin/bash
# K7 flash prefill: numerics, microbench, engine tests; then LLM canaries
source scripts/gpu_check.sh
step pytest_attn 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "attention or flash"
step bench_attn 300 python scripts/bench_attn.py
step pytest_model 600 python -m pytest tests/test_model_gpu.py tests/test_tp_gpu.py -q -m gpu -x
step pytest_canary 900 python -m pytest tests/test_llm_canary_gpu.py -q -m gpu -x
