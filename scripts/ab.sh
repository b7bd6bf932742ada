#!/bin/bash
# Interleaved same-box A/B of the driver's bench command under two settings.
# Usage: gpurun -- bash scripts/ab.sh "A" "B" [ROUNDS] [extra bench.py args...]
#   A / B: words NAME=value with an upper-case NAME are environment variables, anything else is
#   passed to bench.py (e.g. "--ab-ops gemm_half_tile=0"); an empty string = the defaults.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A=$1; B=$2; R=${3:-2}; shift 3 || shift $#
split() {  # $1 -> ENVS / ARGS arrays
  ENVS=(); ARGS=()
  for w in $1; do
    if [[ $w =~ ^[A-Z_][A-Z0-9_]*= ]]; then ENVS+=("$w"); else ARGS+=("$w"); fi
  done
}
for i in $(seq 1 "$R"); do
  split "$A"; step "ab_A$i" 600 env "${ENVS[@]}" python3 bench.py --gpus 1 --steps 20 --warmup 5 --cr-ready-samples 0 "${ARGS[@]}" "$@"
  split "$B"; step "ab_B$i" 600 env "${ENVS[@]}" python3 bench.py --gpus 1 --steps 20 --warmup 5 --cr-ready-samples 0 "${ARGS[@]}" "$@"
done
