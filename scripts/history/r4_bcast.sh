#!/bin/bash
# K15 IPC broadcast of the TP step metadata: GPU tests, a TP=2-on-one-GPU kernel trace (idle gaps
# between steps), the default bench (fresh-process predictor start-up phases).
bash scripts/steps.sh \
  "car 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_custom_ar_gpu.py" \
  "tp 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_tp_gpu.py" \
  "tp2trace 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_tp2 -o tp -- python3 bench.py --gpus 2 --tp 2 --share-gpu --batch 256 --steps 20 --warmup 5 --no-operator" \
  "bench 600 python3 bench.py --gpus 1 --steps 20 --warmup 5"
