#!/bin/bash
# decode graphs without the identity logits-row gather, decode ids gathered by one kernel:
# full GPU suite, then batch 1 / 4 and the headline
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
B="python3 bench.py --steps 100 --warmup 20 --no-operator --cr-ready-samples 0"
bash scripts/steps.sh \
  "suite 900 $T tests" \
  "g1a 300 $B --batch 1" "g4 300 $B --batch 4" "g1b 300 $B --batch 1" \
  "head 600 python3 bench.py --no-operator --cr-ready-samples 0"
