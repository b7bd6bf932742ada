#!/bin/bash
# token-major V A/B (attention kernels, bit-identity + time) and the TP=2-on-one-GPU trace with
# one kernel-trace file per rank process
bash scripts/steps.sh \
  "vt 300 python3 scripts/bench_vt.py" \
  "tp2trace 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_tp2b -o tp_%pid% -- python3 bench.py --gpus 2 --tp 2 --share-gpu --batch 256 --steps 20 --warmup 5 --no-operator"
