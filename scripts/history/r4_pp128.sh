#!/bin/bash
# ping-pong kernel admitted from 128 tiles (new default) vs 192 (MLOP_GEMM_PP_MIN_TILES=192):
# GEMM tests, mid-M microbench, batch 512 / 1024 serving and the headline, interleaved
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
B="python3 bench.py --steps 60 --warmup 10 --no-operator --cr-ready-samples 0"
O="env MLOP_GEMM_PP_MIN_TILES=192"
bash scripts/steps.sh \
  "tp128 600 $T tests/test_kernels_gpu.py tests/test_norm_chain_gpu.py -k 'gemm or chain or rope'" \
  "mbp 600 env BENCH_MS=1536,2304,2560 BENCH_TAG=new python3 scripts/bench_gemm.py" \
  "p512n 500 $B --batch 512" "p512o 500 $O $B --batch 512" \
  "p1kn 500 $B --batch 1024" "p1ko 500 $O $B --batch 1024" \
  "phn 600 python3 bench.py --no-operator --cr-ready-samples 0" "pho 600 $O python3 bench.py --no-operator --cr-ready-samples 0"
