#!/bin/bash
# Decode paged-attention bandwidth at the headline shape (scripts/bench_attn.py).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step attn_b2048 200 python scripts/bench_attn.py
step attn_b256 200 env B=256 CTX=1024,4096 python scripts/bench_attn.py
step attn_b32 200 env B=32 CTX=4096,8192 python scripts/bench_attn.py
