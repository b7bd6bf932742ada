#!/bin/bash
# two-wave K-split GEMV workgroups (KW = 2) at M <= 2: MLOP_GEMV_KW2 0 (off) / 1 (QKV only,
# default) / 2 (every K-split launch); GEMV + chain tests in modes 1 and 2, then batch 1 / 2
# interleaved; MLOP_ATTN_MIN_PART=256 once at batch 1
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
B="python3 bench.py --steps 100 --warmup 20 --no-operator --cr-ready-samples 0"
bash scripts/steps.sh \
  "t1 600 $T tests/test_kernels_gpu.py -k gemv tests/test_norm_chain_gpu.py -k 'gemv or decode'" \
  "t2 600 env MLOP_GEMV_KW2=2 $T tests/test_kernels_gpu.py -k gemv tests/test_norm_chain_gpu.py -k 'gemv or decode'" \
  "k0a 300 env MLOP_GEMV_KW2=0 $B --batch 1" "k1a 300 $B --batch 1" "k2a 300 env MLOP_GEMV_KW2=2 $B --batch 1" \
  "j0 300 env MLOP_GEMV_KW2=0 $B --batch 2" "j1 300 $B --batch 2" "j2 300 env MLOP_GEMV_KW2=2 $B --batch 2" \
  "k0b 300 env MLOP_GEMV_KW2=0 $B --batch 1" "k1b 300 $B --batch 1" "k2b 300 env MLOP_GEMV_KW2=2 $B --batch 1" \
  "mp256 300 env MLOP_ATTN_MIN_PART=256 $B --batch 1"
