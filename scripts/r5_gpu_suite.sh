#!/bin/bash
# the round-end driver sequence, early: the whole GPU suite, smoke(), then the cold small-M sweep
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step gpu_suite 1100 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step smallm_cold 400 python -u scripts/bench_small_m.py
