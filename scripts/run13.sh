#!/bin/bash
source scripts/gpu_check.sh
step pytest_canary 900 python -m pytest tests/test_llm_canary_gpu.py -q -m gpu -x
