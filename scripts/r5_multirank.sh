#!/bin/bash
# one-GPU rehearsals of the multi-rank paths on the final tree (TP = 2, EP = 2, both ranks on device 0)
source scripts/gpu_check.sh
step tp2 500 python3 bench.py --gpus 2 --tp 2 --share-gpu --batch 256 --steps 20 --warmup 5 --no-operator
step ep2 500 python3 bench.py --gpus 2 --ep 2 --share-gpu --model mixtral-8x7b --batch 256 --steps 30 --warmup 5 --kv-gb 40 --no-operator
