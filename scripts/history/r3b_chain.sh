#!/bin/bash
# Norm chain (O / down add into the residual with row partials; gate_up / QKV scale rows after the
# GEMM): numerics, the GEMM / model suites it touches, then the driver command chain on vs off.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step t_chain 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_norm_chain_gpu.py tests/test_gemm_w4_gpu.py tests/test_model_gpu.py
B="python3 bench.py --gpus 1 --steps 20 --warmup 5"
step d_on_a 400 $B
step d_off_a 400 env MLOP_NORM_CHAIN=0 $B
step d_on_b 400 $B
step d_off_b 400 env MLOP_NORM_CHAIN=0 $B
