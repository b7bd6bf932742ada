#!/bin/bash
source scripts/gpu_check.sh
step prof_bench 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o bench --output-format csv -- python3 bench.py --steps 100 --warmup 30
