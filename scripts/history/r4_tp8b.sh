#!/bin/bash
# TP = 8 on one GPU with Llama-3-8B (one kv head per rank) and start-up progress lines, to see
# where the 70B run of r4_tp8.sh spent its silent minutes
MLOP_VERBOSE=1 bash scripts/steps.sh \
  "tp8s 500 python3 bench.py --gpus 8 --tp 8 --share-gpu --model llama3-8b --batch 64 --steps 10 --warmup 3 --kv-gb 8 --no-operator"
