#!/bin/bash
# fused split-KV combine on by default: race tests + attention tests, then the headline bench
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
bash scripts/steps.sh \
  "races 400 $T tests/test_races_gpu.py" \
  "attn 400 $T tests/test_kernels_gpu.py -k attention" \
  "head 600 python3 bench.py --no-operator --cr-ready-samples 0"
