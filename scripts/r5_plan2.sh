#!/bin/bash
# Dead A rows as dropped out-of-range DMA in the ping-pong kernel: GEMM numerics, the MoE
# spill counts, Mixtral batch 1024, then the headline under the round-5 vs round-4 planner x3
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step gemmtests2 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_w4_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm or grouped or moe or engine"
step moecnt2 600 python -u scripts/bench_moe_decode.py --counts '256,256,256,256,256,256,256,256;257,257,257,257,257,257,257,257;248,237,278,267,251,264,261,242'
step mix1024 500 python3 bench.py --no-operator --model mixtral-8x7b --batch 1024 --steps 30 --warmup 10
for i in 1 2 3; do
  step "hnew_$i" 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cr-ready-samples 0
  step "hold_$i" 500 env MLOP_GEMM_PLAN_R4=1 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cr-ready-samples 0
done
