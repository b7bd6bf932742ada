#!/bin/bash
# Prefill-heavy serving after the flash prefill work (before: scripts/run99.sh, 75.4k prefill tok/s), + default bench.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pf_bench 600 python bench.py --no-operator --batch 256 --prompt-len 2048 --output-len 32 --max-model-len 4096 --steps 60 --warmup 20
step bench 600 python bench.py
