#!/bin/bash
# Decode tiles in descending context order (LPT) vs row order, same box, alternating.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step bench_lpt 600 python bench.py --no-operator
step bench_rows 600 env MLOP_DECODE_LPT=0 python bench.py --no-operator
step bench_lpt2 600 python bench.py --no-operator
step bench_rows2 600 env MLOP_DECODE_LPT=0 python bench.py --no-operator
