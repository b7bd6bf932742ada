#!/bin/bash
# Split-K target of the row-fitted small-M tiles (workgroups per narrow projection), cold op level.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for t in 256 512 1024; do
  step split_$t 200 env MLOP_GEMM_SPLIT_TARGET=$t WSG_MIN_WG= SMALL_TILES=64 BENCH_MS=8,16,32,64 python scripts/bench_wsg.py
done
