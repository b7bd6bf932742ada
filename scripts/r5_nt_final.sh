#!/bin/bash
# nt-weights / nt-KV defaults on the final tree: the whole GPU suite, smoke(), the driver's bench
# command, then the batch rows of BASELINE.md
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step gpu_suite 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step driver 500 python3 bench.py --gpus 1 --steps 20 --warmup 5
for b in 16 64 256; do
  step "llama_b$b" 300 python3 bench.py --no-operator --batch $b --steps 60 --warmup 10 --cr-ready-samples 0
done
for b in 64 256 1024; do
  step "mixtral_b$b" 400 python3 bench.py --no-operator --model mixtral-8x7b --batch $b --steps 30 --warmup 10 --cr-ready-samples 0
done
