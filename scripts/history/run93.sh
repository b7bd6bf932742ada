#!/bin/bash
# Decode attention: forced partition lengths at long contexts (scripts/bench_attn.py PART=...).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in "256 1024,4096" "32 4096,8192" "64 2048,8192" "2048 256,512"; do
  set -- $cfg
  for part in "" 512 1024 2048; do
    step attn_${1}_${part:-auto} 200 env B=$1 CTX=$2 PART=$part python scripts/bench_attn.py
  done
done
