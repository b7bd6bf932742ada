#!/bin/bash
# the driver's command three times: HTTP-served rate on the engine clock vs the client window
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2 3; do
  step "drv$i" 500 python3 bench.py --gpus 1 --steps 20 --warmup 5
done
