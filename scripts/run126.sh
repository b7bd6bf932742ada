#!/bin/bash
# Calibration: the M <= 4 GEMV (1-KiB contiguous runs per load instruction) on the same
# rotating-weights harness as the mid-size arms of run125.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step gemv_cal 200 env BENCH_MS=1,4,8 WSG_MIN_WG=128 python scripts/bench_wsg.py
step gemv8_cal 200 env MLOP_GEMV_MAX_M=8 BENCH_MS=8 WSG_MIN_WG=128 python scripts/bench_wsg.py
