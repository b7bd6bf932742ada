#!/bin/bash
# confirmation rounds: defaults vs both output-store nt options on the headline
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2 3; do
  step "base$i" 500 python3 bench.py --no-operator --steps 20 --warmup 5 --cr-ready-samples 0
  step "both$i" 500 python3 bench.py --no-operator --steps 20 --warmup 5 --cr-ready-samples 0 --ab-ops gemm_slab_nt=15,attn_kv_nt=3
done
