#!/bin/bash
source scripts/gpu_check.sh
step pytest_gpu 900 python -m pytest tests -q -m gpu -x
step bench 900 python bench.py
