#!/bin/bash
# Round-2 re-entry check on a fresh box: the full GPU suite (as the driver runs it), smoke(),
# then the default headline bench.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 500 python bench.py
