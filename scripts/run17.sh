#!/bin/bash
# GEMM choice table: measure it fresh, then start-up + bench with it
source scripts/gpu_check.sh
step b_tune 600 env MLOP_GEMM_TABLE=off python bench.py --steps 60 --warmup 40 --save-gemm-table gpurun_out/gemm_table_gfx950.json
cp gpurun_out/gemm_table_gfx950.json research-and-development-of-kubernetes-operator-for-machine-learning-pipelines_amd/ops/gemm_table_gfx950.json
step b_table 600 python bench.py --steps 100 --warmup 40
step pytest_model 600 python -m pytest tests/test_model_gpu.py -q -m gpu -x
