#!/bin/bash
# decode attention at 4 waves per SIMD (127 VGPRs, default) vs 3 (134 VGPRs, MLOP_ATTN_WPE=1):
# race + attention tests (the earlier fused-combine change too), then decode-attention microbench
# and the headline bench, interleaved on one box
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
H="python3 bench.py --no-operator --cr-ready-samples 0"
bash scripts/steps.sh \
  "races 400 $T tests/test_races_gpu.py" \
  "attn 400 $T tests/test_kernels_gpu.py -k attention" \
  "o4a 300 python3 scripts/bench_decode_attn.py" \
  "o3a 300 env MLOP_ATTN_WPE=1 python3 scripts/bench_decode_attn.py" \
  "o4b 300 python3 scripts/bench_decode_attn.py" \
  "o3b 300 env MLOP_ATTN_WPE=1 python3 scripts/bench_decode_attn.py" \
  "h4a 600 $H" "h3a 600 env MLOP_ATTN_WPE=1 $H" "h4b 600 $H" "h3b 600 env MLOP_ATTN_WPE=1 $H"
