#!/bin/bash
# Round-3 re-entry baseline: GEMM A/B at the headline shapes, GPU tests, smoke, default bench.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step gemm_ab 300 python -u scripts/bench_bigm.py
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python -u bench.py
