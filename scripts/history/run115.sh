#!/bin/bash
# TunableOp (exhaustive hipBLASLt / rocBLAS solution search per exact shape) vs torch.matmul's
# default pick and the hand-written ping-pong kernel, at the headline's row counts.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step tunable 900 python -u scripts/bench_tunable.py
