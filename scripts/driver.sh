#!/bin/bash
# The driver's round-end sequence on one box: GPU suite, smoke(), then the driver's bench
# command REPEAT times (default 2).  Usage: gpurun -- bash scripts/driver.sh [REPEAT] [--no-tests]
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
REPEAT=${1:-2}
if [ "${2:-}" != "--no-tests" ]; then
  step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
for i in $(seq 1 "$REPEAT"); do
  step "bench_driver$i" 600 python3 bench.py --gpus 1 --steps 20 --warmup 5
done
