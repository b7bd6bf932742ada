#!/bin/bash
# The driver's round-end sequence on one box: GPU suite, smoke, then its bench command.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_driver 600 python3 bench.py --gpus 1 --steps 20 --warmup 5
step bench_driver2 600 python3 bench.py --gpus 1 --steps 20 --warmup 5
