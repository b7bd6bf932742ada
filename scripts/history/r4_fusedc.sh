#!/bin/bash
# split-KV combine in-launch with sc1 partial stores (no producer release fence): attention
# tests + race test, then batch 1 / 8 / 16 / 64 with the fused-pair cap at 32 (default) vs
# unlimited, interleaved on one box
B="python3 bench.py --steps 100 --warmup 20 --no-operator --cr-ready-samples 0"
U="env MLOP_ATTN_FUSED_MAX_PAIRS=1000000"
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
bash scripts/steps.sh \
  "tests 400 $T tests/test_kernels_gpu.py -k paged_attention tests/test_races_gpu.py" \
  "b1_d 300 $B --batch 1" "b1_u 300 $U $B --batch 1" \
  "b8_d 300 $B --batch 8" "b8_u 300 $U $B --batch 8" \
  "b16_d 300 $B --batch 16" "b16_u 300 $U $B --batch 16" \
  "b64_d 300 $B --batch 64" "b64_u 300 $U $B --batch 64" \
  "b1_d2 300 $B --batch 1" "b1_u2 300 $U $B --batch 1"
