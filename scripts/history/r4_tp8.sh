#!/bin/bash
# TP = 8 rehearsed on one GPU: the 8-rank K15 kernels (test), then Llama-3-70B TP = 8 through
# bench.py with 8 rank processes sharing the card (gloo + IPC collectives, shm header ring with
# 7 consumers): a correctness / path rehearsal of config 4, not a performance number
bash scripts/steps.sh \
  "car8 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_custom_ar_gpu.py" \
  "tp8 900 python3 bench.py --gpus 8 --tp 8 --share-gpu --model llama3-70b --batch 64 --steps 10 --warmup 3 --kv-gb 8 --no-operator"
