#!/bin/bash
# planner by tile count: large-M kernels from 512 rows at >= 72 tiles of 256x256, the 256x128
# kernel below 72 tiles up to 2048 rows (new default) vs the old plan (large-M kernels from 1024
# rows everywhere: MLOP_GEMM_BIG_WIDE_MIN_M=1024 MLOP_GEMM_BIG_MID_TILES=0); tests, then batch
# 512 / 768 / 1024 serving and the headline, interleaved
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
B="python3 bench.py --steps 60 --warmup 10 --no-operator --cr-ready-samples 0"
O="env MLOP_GEMM_BIG_WIDE_MIN_M=1024 MLOP_GEMM_BIG_MID_TILES=0"
bash scripts/steps.sh \
  "tg2 600 $T tests/test_kernels_gpu.py tests/test_norm_chain_gpu.py -k 'gemm or chain or rope'" \
  "v512n 600 $B --batch 512" "v512o 600 $O $B --batch 512" \
  "v768n 600 $B --batch 768" "v768o 600 $O $B --batch 768" \
  "v1kn 600 $B --batch 1024" "v1ko 600 $O $B --batch 1024" \
  "v1kn2 600 $B --batch 1024" "v1ko2 600 $O $B --batch 1024" \
  "hn 600 python3 bench.py --no-operator --cr-ready-samples 0" "ho 600 $O python3 bench.py --no-operator --cr-ready-samples 0"
