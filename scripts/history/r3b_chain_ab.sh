#!/bin/bash
# Norm chain on / off, interleaved on one box, 100 timed steps each (3 pairs).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --gpus 1 --steps 100 --warmup 10"
for i in 1 2 3; do
  step ab_on_$i 400 $B
  step ab_off_$i 400 env MLOP_NORM_CHAIN=0 $B
done
