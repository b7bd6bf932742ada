#!/bin/bash
# MoE decode dispatch: router row + norm weights issued before the prologue, normalised rows
# staged in LDS for the router and the gather; MoE tests, then Mixtral batch 1 / 4 against the
# previous commit's build (a worktree under build/abold), interleaved
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
B="python3 bench.py --model mixtral-8x7b --steps 60 --warmup 10 --no-operator --cr-ready-samples 0"
bash scripts/steps.sh \
  "tm 600 $T tests/test_kernels_gpu.py -k 'moe or dispatch or mixtral'" \
  "d1n 400 $B --batch 1" "d1o 400 bash -c 'cd build/abold && $B --batch 1'" \
  "d4n 400 $B --batch 4" "d4o 400 bash -c 'cd build/abold && $B --batch 4'" \
  "d1n2 400 $B --batch 1" "d1o2 400 bash -c 'cd build/abold && $B --batch 1'"
