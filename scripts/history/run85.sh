#!/bin/bash
# Projection alternatives at the headline's row counts (scripts/bench_proj.py).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step bench_proj 500 python scripts/bench_proj.py
