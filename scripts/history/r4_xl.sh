#!/bin/bash
# GEMV activations staged in LDS once per workgroup at 3-4 rows (XL, default) vs each wave
# re-reading them (MLOP_GEMV_XL=0): GEMV / chain / race tests, then batch 3 / 4 interleaved
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
B="python3 bench.py --steps 100 --warmup 20 --no-operator --cr-ready-samples 0"
bash scripts/steps.sh \
  "tx 600 $T tests/test_kernels_gpu.py tests/test_norm_chain_gpu.py tests/test_races_gpu.py -k 'gemv or norm or chain or decode'" \
  "x4a 300 $B --batch 4" "n4a 300 env MLOP_GEMV_XL=0 $B --batch 4" \
  "x3 300 $B --batch 3" "n3 300 env MLOP_GEMV_XL=0 $B --batch 3" \
  "x4b 300 $B --batch 4" "n4b 300 env MLOP_GEMV_XL=0 $B --batch 4"
