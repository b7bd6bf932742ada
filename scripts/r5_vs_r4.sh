#!/bin/bash
# same-box A/B of the round-4 tree (git worktree at build/r4tree, its own extension) against
# this tree at small batch
source scripts/gpu_check.sh
R=$GRAFT_REPO_ROOT
for b in 4 16 64; do
  for i in 1 2; do
    step "r5_b${b}_$i" 300 python3 bench.py --no-operator --batch $b --steps 60 --warmup 10 --cr-ready-samples 0
    cd "$R/build/r4tree" && step_dir=1
    timeout -k 10 300 python3 bench.py --no-operator --batch $b --steps 60 --warmup 10 --cr-ready-samples 0 > "$R/gpurun_out/r4_b${b}_$i.log" 2>&1
    rc=$?; cd "$R"; echo "== r4_b${b}_$i rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  done
done
