#!/bin/bash
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step normtests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "rmsnorm" --timeout 120 --timeout-method thread
step norm_new 120 python -u scripts/bench_norm.py
step norm_old 120 env NORM_LIB=build/norm_ab/_C_norm_old.so python -u scripts/bench_norm.py
step norm_new2 120 python -u scripts/bench_norm.py
