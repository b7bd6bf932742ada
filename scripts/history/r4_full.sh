#!/bin/bash
# round-4 tree on one box: the driver's sequence (GPU suite, smoke, driver bench x2), then the
# TP=2 and EP=2 one-GPU rehearsals of the multi-rank paths
bash scripts/driver.sh 2 && bash scripts/steps.sh \
  "tp2 600 python3 bench.py --gpus 2 --tp 2 --share-gpu --batch 256 --steps 20 --warmup 5 --no-operator" \
  "ep2 900 python3 bench.py --gpus 2 --ep 2 --share-gpu --model mixtral-8x7b --batch 256 --steps 30 --warmup 5 --kv-gb 40 --no-operator"
