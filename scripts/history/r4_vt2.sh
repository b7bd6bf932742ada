#!/bin/bash
# token-major V everywhere + IPC all-gather: the GPU suite, then the TP=2-on-one-GPU trace (one
# kernel-trace file per rank process) for the idle-gap analysis (scripts/trace_window.py --by-pid)
bash scripts/steps.sh \
  "gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "tp2trace 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_tp2c -o tp_%pid% -- python3 bench.py --gpus 2 --tp 2 --share-gpu --batch 256 --steps 20 --warmup 5 --no-operator"
