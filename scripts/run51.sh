#!/bin/bash
# Wave-per-row RMSNorm: numerics at many-row shapes, then default bench with it on/off.
source scripts/gpu_check.sh
cd "$GRAFT_REPO_ROOT"
step norm_tests 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "rmsnorm" --timeout 120 --timeout-method thread
step bench_wave 400 python bench.py --steps 100 --warmup 20 --no-operator
MLOP_NORM_WAVE=0 step bench_nowave 400 python bench.py --steps 100 --warmup 20 --no-operator
