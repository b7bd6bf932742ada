#!/bin/bash
# non-temporal q / K / V stores of the four-wave RoPE epilogue (gemm_slab_nt bit 3) and of the
# decode attention output (attn_kv_nt 3): headline A/B, numerics first
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_norm_chain_gpu.py tests/test_kernels_gpu.py -k "rope or attention or chain"
for i in 1 2; do
  step "base$i" 500 python3 bench.py --no-operator --steps 20 --warmup 5 --cr-ready-samples 0
  step "rope$i" 500 python3 bench.py --no-operator --steps 20 --warmup 5 --cr-ready-samples 0 --ab-ops gemm_slab_nt=15
  step "attn$i" 500 python3 bench.py --no-operator --steps 20 --warmup 5 --cr-ready-samples 0 --ab-ops attn_kv_nt=3
  step "both$i" 500 python3 bench.py --no-operator --steps 20 --warmup 5 --cr-ready-samples 0 --ab-ops gemm_slab_nt=15,attn_kv_nt=3
done
