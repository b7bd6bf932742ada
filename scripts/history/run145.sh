#!/bin/bash
# gate_up at M 33-64 (64 x 64 tiles): ring depth 3 vs 4 vs 6, cold op level.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step gu64 200 env WSG_MIN_WG= SMALL_TILES=1 SMALL_STAGES=3,4,6 BENCH_MS=40,48,64 python scripts/bench_wsg.py
