#!/bin/bash
# Full GPU suite + smoke + default bench (driver form) + batch 1 / 64 on the current tree.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step gputests142 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke142 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench142 500 python bench.py --steps 20 --warmup 5
step b1_142 200 python bench.py --batch 1 --steps 200 --warmup 20 --no-operator
step b64_142 200 python bench.py --batch 64 --steps 150 --warmup 20 --no-operator
