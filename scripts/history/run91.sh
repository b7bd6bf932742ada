#!/bin/bash
# Concurrency sweep of the headline config (same box): 2048 (default) vs 2560 vs 3072.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step bench_b2048 600 python bench.py --no-operator
step bench_b2560 600 python bench.py --no-operator --batch 2560
step bench_b3072 600 python bench.py --no-operator --batch 3072
