#!/bin/bash
# Round-5 planner rules (grouped ping-pong from 56 rows per expert, long-K mid-M on the
# ping-pong kernel, four-wave vs ping-pong round model): GEMM numerics first, then the
# same-box interleaved A/B against the round-4 rules (MLOP_GEMM_PLAN_R4=1)
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step gemmtests 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_w4_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm or grouped or moe"
for cfg in "--batch 512 --steps 60 --warmup 10" "--batch 1024 --steps 60 --warmup 10" "--model mixtral-8x7b --batch 256 --steps 30 --warmup 10" "--model mixtral-8x7b --batch 1024 --steps 30 --warmup 10"; do
  tag=$(echo "$cfg" | tr -cd 'a-z0-9' | cut -c1-24)
  for i in 1 2; do
    step "new_${tag}_$i" 500 python3 bench.py --no-operator $cfg
    step "old_${tag}_$i" 500 env MLOP_GEMM_PLAN_R4=1 python3 bench.py --no-operator $cfg
  done
done
step "new_head" 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cr-ready-samples 0
step "old_head" 500 env MLOP_GEMM_PLAN_R4=1 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cr-ready-samples 0
