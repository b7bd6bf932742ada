#!/bin/bash
# Generic runner: each argument is "NAME TIMEOUT CMD..." (one GPU step, own time limit, logged to
# gpurun_out/NAME.log, the script stops at the first crash or timeout).
# Usage: gpurun -- bash scripts/steps.sh "t1 300 python -m pytest tests/test_x.py -m gpu" "b 600 python3 bench.py"
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for spec in "$@"; do
  eval "step $spec"  # eval: quotes inside a spec group words ("-c 'import x; x.f()'")
done
