#!/bin/bash
source scripts/gpu_check.sh
step prof_bench 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 10 --no-operator
ls -R gpurun_out/prof | head -20
