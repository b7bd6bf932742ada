#!/bin/bash
# Two-level ticket GEMV add+norm epilogue: numerics, then batch-1 decode A/B (epilogue on/off, lazy KV on/off).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_addnorm 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "add_rmsnorm"
step b1 300 python bench.py --batch 1 --steps 300 --warmup 20 --no-operator
MLOP_GEMV_ADDNORM=0 step b1_noaddnorm 300 python bench.py --batch 1 --steps 300 --warmup 20 --no-operator
MLOP_GEMV_ADDNORM=0 MLOP_KV_LAZY=0 step b1_noaddnorm_eagerkv 300 python bench.py --batch 1 --steps 300 --warmup 20 --no-operator
step b4 300 python bench.py --batch 4 --steps 300 --warmup 20 --no-operator
