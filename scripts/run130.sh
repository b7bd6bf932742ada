#!/bin/bash
# Full GPU suite + smoke + default bench on the current tree (wsgemm off by default).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step gputests130 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke130 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench130 500 python bench.py --steps 20 --warmup 5
