#!/bin/bash
# GEMV with the residual add + RMSNorm in a last-ticket epilogue: numerics, then batch-1..4 decode.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_addnorm 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "add_rmsnorm"
step pytest_model 300 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread
step b1 300 python bench.py --batch 1 --steps 300 --warmup 20 --no-operator
step b2 300 python bench.py --batch 2 --steps 300 --warmup 20 --no-operator
step b4 300 python bench.py --batch 4 --steps 300 --warmup 20 --no-operator
