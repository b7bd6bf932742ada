#!/bin/bash
# Interleaved same-box A/B of the driver's bench command under two environments.
# Usage: gpurun -- bash scripts/ab.sh "ENV_A=1" "ENV_B=0" [ROUNDS] [extra bench.py args...]
#        (an empty string = the default environment)
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A=$1; B=$2; R=${3:-2}; shift 3 || shift $#
for i in $(seq 1 "$R"); do
  step "ab_A$i" 600 env $A python3 bench.py --gpus 1 --steps 20 --warmup 5 --cr-ready-samples 0 "$@"
  step "ab_B$i" 600 env $B python3 bench.py --gpus 1 --steps 20 --warmup 5 --cr-ready-samples 0 "$@"
done
