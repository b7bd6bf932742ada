#!/bin/bash
# TP decode norm chain (all-reduce + residual add in one K15 launch, row-scaled GEMVs):
# collectives + TP + chain GPU tests, then Llama-3-8B TP = 2 and TP = 8 on one GPU at batch 4
# (time-sliced: a functional end-to-end run, not a speed number), chain on vs MLOP_GEMV_CHAIN=0
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
B="python3 bench.py --share-gpu --model llama3-8b --batch 4 --steps 20 --warmup 5 --no-operator --cr-ready-samples 0"
bash scripts/steps.sh \
  "car 600 $T tests/test_custom_ar_gpu.py" \
  "tp 600 $T tests/test_tp_gpu.py tests/test_norm_chain_gpu.py" \
  "tp2c 400 $B --gpus 2 --tp 2" "tp2n 400 env MLOP_GEMV_CHAIN=0 $B --gpus 2 --tp 2" \
  "tp8c 500 $B --gpus 8 --tp 8 --kv-gb 8"
