#!/bin/bash
# M = 128 / 256 projections: ring depth of the 128-row tile (3 vs 5) vs hipBLASLt, cold op level.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step m128 300 env WSG_MIN_WG= SMALL_TILES=1 SMALL_STAGES=3,5 BENCH_MS=96,128,256 python scripts/bench_wsg.py
