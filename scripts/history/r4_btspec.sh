#!/bin/bash
# decode attention reads the wave's first page pair in the same round trip as ctx_len (block
# table speculation): attention + race tests, decode-attention microbench, batch 1 / 8 benches
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
B="python3 bench.py --steps 100 --warmup 20 --no-operator --cr-ready-samples 0"
bash scripts/steps.sh \
  "races 400 $T tests/test_races_gpu.py" \
  "attn 400 $T tests/test_kernels_gpu.py -k attention" \
  "da 300 python3 scripts/bench_decode_attn.py" \
  "b1a 300 $B --batch 1" "b8a 300 $B --batch 8" "b1b 300 $B --batch 1" "b8b 300 $B --batch 8"
