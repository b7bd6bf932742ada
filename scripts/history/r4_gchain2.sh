#!/bin/bash
# full GPU suite after the GEMV chain, then the headline bench and batch 1
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
bash scripts/steps.sh \
  "suite 900 $T tests" \
  "head 600 python3 bench.py --no-operator --cr-ready-samples 0" \
  "b1 300 python3 bench.py --steps 100 --warmup 20 --no-operator --cr-ready-samples 0 --batch 1"
