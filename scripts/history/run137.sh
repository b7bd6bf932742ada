#!/bin/bash
# BM 16 small-M tiles: BN 32 / 64 x ring depth 4 / 6 / 8 (bytes in flight per CU), cold op level.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step bn_stg 300 env WSG_MIN_WG= SMALL_TILES=32,64 SMALL_STAGES=3,6,8 BENCH_MS=8,16 python scripts/bench_wsg.py
