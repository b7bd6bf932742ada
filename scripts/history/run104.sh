#!/bin/bash
# Decode attention: same KV bytes (~1 GB), different (batch, context) splits, fixed contexts.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in "2048 256,256" "512 1024,1024" "128 4096,4096" "64 8192,8192" "32 16384,16384"; do
  set -- $cfg
  step attn_${1} 200 env B=$1 CTX=$2 python scripts/bench_attn.py
done
step attn_64_p1024 200 env B=64 CTX=8192,8192 PART=1024 python scripts/bench_attn.py
step attn_64_p2048 200 env B=64 CTX=8192,8192 PART=2048 python scripts/bench_attn.py
