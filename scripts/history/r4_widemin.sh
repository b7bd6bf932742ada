#!/bin/bash
# large-M kernels for wide grids from 512 rows (MLOP_GEMM_BIG_WIDE_MIN_M=512, new default) vs
# from 1024 (=1024, the old plan): GEMM tests, microbench, then batch 512 / 1024 serving, interleaved
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
B="python3 bench.py --steps 60 --warmup 10 --no-operator --cr-ready-samples 0"
O="env MLOP_GEMM_BIG_WIDE_MIN_M=1024"
bash scripts/steps.sh \
  "tg 600 $T tests/test_kernels_gpu.py tests/test_norm_chain_gpu.py -k 'gemm or chain or rope'" \
  "mb 600 env BENCH_MS=512,768 BENCH_TAG=new python3 scripts/bench_gemm.py" \
  "w512n 600 $B --batch 512" "w512o 600 $O $B --batch 512" \
  "w1kn 600 $B --batch 1024" "w1ko 600 $O $B --batch 1024" \
  "w512n2 600 $B --batch 512" "w512o2 600 $O $B --batch 512"
