#!/bin/bash
# grouped small-tile sweep at batch 32 / 64 routing (64 / 128 routed rows over 8 experts)
source scripts/gpu_check.sh
step moesm 400 python -u scripts/bench_moe_decode.py --rows 64,128 --iters 10
