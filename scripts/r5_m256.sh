#!/bin/bash
# decode-sized M = 128-256 (batch 128-256 serving) projection tilings with cold weights
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step m256 600 python3 scripts/bench_mid_m.py --cold --ms 256,192,128 --iters 10
