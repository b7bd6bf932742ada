#!/bin/bash
# Full GPU suite + smoke + default bench after the MoE prologue / prefix cache / loader work.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
