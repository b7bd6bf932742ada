#!/bin/bash
# Full GPU suite + smoke + the driver's bench command on one box.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step drv1 400 python3 bench.py --gpus 1 --steps 20 --warmup 5
step drv2 400 python3 bench.py --gpus 1 --steps 20 --warmup 5
