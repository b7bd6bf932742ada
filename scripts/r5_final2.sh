#!/bin/bash
# round-end rehearsal on the final tree: the whole GPU suite, smoke(), the driver's bench command
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step gpu_suite 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step driver 500 python3 bench.py --gpus 1 --steps 20 --warmup 5
