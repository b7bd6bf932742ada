#!/bin/bash
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step rope_var 300 python -u scripts/bench_rope_var.py
