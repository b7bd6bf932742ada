#!/bin/bash
# Full GPU suite with the lazily backed KV arena as the default, smoke.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 300 python __graft_entry__.py smoke
