#!/bin/bash
source scripts/gpu_check.sh
step pytest_tp 600 python -m pytest tests/test_tp_gpu.py -q -m gpu -x
