#!/bin/bash
# decode norm chain on the GEMV (EPI_RES / PRO_RS): chain tests + GEMV / engine tests, then
# batch 1 / 2 / 4 with the chain (default) vs MLOP_GEMV_CHAIN=0, interleaved on one box
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
B="python3 bench.py --steps 100 --warmup 20 --no-operator --cr-ready-samples 0"
bash scripts/steps.sh \
  "chain 600 $T tests/test_norm_chain_gpu.py" \
  "gemv 600 $T tests/test_kernels_gpu.py -k 'gemv or norm'" \
  "b1c 300 $B --batch 1" "b1n 300 env MLOP_GEMV_CHAIN=0 $B --batch 1" \
  "b2c 300 $B --batch 2" "b2n 300 env MLOP_GEMV_CHAIN=0 $B --batch 2" \
  "b4c 300 $B --batch 4" "b4n 300 env MLOP_GEMV_CHAIN=0 $B --batch 4" \
  "b1c2 300 $B --batch 1" "b1n2 300 env MLOP_GEMV_CHAIN=0 $B --batch 1"
