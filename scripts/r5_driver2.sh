#!/bin/bash
# the driver's bench command twice (engine-direct and HTTP-served rates), nt defaults
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step driver_a 500 python3 bench.py --gpus 1 --steps 20 --warmup 5
step driver_b 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 --ab-ops attn_kv_nt=0,gemm_small_nt=0
step driver_c 500 python3 bench.py --gpus 1 --steps 20 --warmup 5
