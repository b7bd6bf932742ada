#!/bin/bash
# RoPE slab kernel over 2 blocks per token A/B at batch 16 / 64 (the rope_split op it flipped was removed
# after this run: two blocks are now fixed), after the GPU suite, smoke() and the driver's command
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step gpu_suite 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step driver 500 python3 bench.py --gpus 1 --steps 20 --warmup 5
for i in 1 2; do
  for b in 64 16; do
    step "b${b}_s1_$i" 300 python3 bench.py --no-operator --batch $b --steps 60 --warmup 10 --cr-ready-samples 0 --ab-ops rope_split=1
    step "b${b}_s2_$i" 300 python3 bench.py --no-operator --batch $b --steps 60 --warmup 10 --cr-ready-samples 0
  done
done
