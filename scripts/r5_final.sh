#!/bin/bash
# round-end rehearsal of the driver sequence on the final tree: the whole GPU suite, smoke(),
# the driver's bench command, then long-context rows for BASELINE.md
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step gpu_suite 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step driver 500 python3 bench.py --gpus 1 --steps 20 --warmup 5
step long32k 500 python3 bench.py --no-operator --model llama3.1-8b --batch 16 --prompt-len 32000 --output-len 256 --max-model-len 32768 --steps 100 --warmup 10 --cr-ready-samples 0
