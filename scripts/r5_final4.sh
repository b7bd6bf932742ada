#!/bin/bash
# last rehearsal of the round on the final tree: GPU suite, smoke(), the driver's command, then
# batch 16 / 64 / 256 and Mixtral batch 64 rows
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step gpu_suite 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step driver 500 python3 bench.py --gpus 1 --steps 20 --warmup 5
for b in 16 64 256; do
  step "fin_b$b" 300 python3 bench.py --no-operator --batch $b --steps 60 --warmup 10 --cr-ready-samples 0
done
step fin_mix64 400 python3 bench.py --no-operator --model mixtral-8x7b --batch 64 --steps 30 --warmup 10 --cr-ready-samples 0
