#!/bin/bash
# served path end to end with the decode norm chain: operator -> fresh predictor process -> V2
# HTTP -> Router, batch 4 (GEMV chain) and batch 256; chain tests incl. the padded batch-3 bucket
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
bash scripts/steps.sh \
  "chain 600 $T tests/test_norm_chain_gpu.py" \
  "h4 600 python3 bench.py --http --batch 4 --steps 20 --warmup 5" \
  "h256 600 python3 bench.py --http --batch 256 --steps 20 --warmup 5"
