#!/bin/bash
# Final validation of the session's tree: GPU suite, smoke, default bench, batch 64.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step gputests146 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke146 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench146 500 python bench.py --steps 20 --warmup 5
step b64_146 200 python bench.py --batch 64 --steps 150 --warmup 20 --no-operator
