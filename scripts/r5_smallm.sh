#!/bin/bash
# small-M tiling sweep (batch 5-64 decode projections) and Mixtral windows at batch 64 / 1024
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step smallm 400 python -u scripts/bench_small_m.py
bash scripts/window.sh mix64 20 --model mixtral-8x7b --batch 64
bash scripts/window.sh mix1024 20 --model mixtral-8x7b --batch 1024
