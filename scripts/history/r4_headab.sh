#!/bin/bash
# headline A/B on one box: this tree vs the round's session-start commit (4502809, a worktree
# under build/abold with its own _C.so), interleaved x2, batch 1 once each
H="python3 bench.py --no-operator --cr-ready-samples 0"
B1="python3 bench.py --steps 100 --warmup 20 --no-operator --cr-ready-samples 0 --batch 1"
bash scripts/steps.sh \
  "hn1 600 $H" "ho1 600 bash -c 'cd build/abold && $H'" \
  "hn2 600 $H" "ho2 600 bash -c 'cd build/abold && $H'" \
  "b1n 300 $B1" "b1o 300 bash -c 'cd build/abold && $B1'"
