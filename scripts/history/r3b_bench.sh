#!/bin/bash
# Default bench + GPU test suite (regression check after a kernel change).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step bench 600 python -u bench.py
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
