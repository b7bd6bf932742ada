#!/bin/bash
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step tests_vdirect 300 env MLOP_V_STAGE=0 python -u -m pytest tests/test_gemm_w4_gpu.py tests/test_kernels_gpu.py -x -q -k rope --timeout 120 --timeout-method thread
step rope_stage 300 python -u scripts/bench_rope_var.py
step rope_direct 300 env MLOP_V_STAGE=0 python -u scripts/bench_rope_var.py
step bench_stage 500 python -u bench.py --steps 100 --warmup 30 --no-operator
step bench_direct 500 env MLOP_V_STAGE=0 python -u bench.py --steps 100 --warmup 30 --no-operator
