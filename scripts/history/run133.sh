#!/bin/bash
# Ring depth of the row-fitted small-M tiles: 4 (default) vs 6 vs 8 stages, cold op level.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step stg_tests 300 env MLOP_GEMM_SMALL_STAGES=8 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "small_tiles and 64"
step stg_bench 300 env WSG_MIN_WG= SMALL_TILES=64 SMALL_STAGES=3,6,8 BENCH_MS=8,16,32,64 python scripts/bench_wsg.py
