#!/bin/bash
# decode attention with double-buffered V images (one pair ahead per wave): attention tests,
# decode / flash microbenches (compare profiles/r04_token_major_v.md), Infinity Cache prefetch probe
bash scripts/steps.sh \
  "kt2 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_races_gpu.py tests/test_model_gpu.py" \
  "dattn 300 python3 scripts/bench_decode_attn.py" \
  "mall 300 python3 scripts/bench_mall.py"
