#!/bin/bash
# The driver's round-end order (GPU suite, smoke, bench) with the bench now waiting for the
# lazily backed KV pool before its ramp (kv_fill_ms / kv_fill_wait_ms in "deploy").
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
step bench2 600 python bench.py
