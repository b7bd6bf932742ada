#!/bin/bash
# Nano-batch two-stream overlap feasibility (scripts/bench_overlap.py).
source scripts/gpu_check.sh
step overlap_a 300 python scripts/bench_overlap.py
M=2048 B=1024 step overlap_b 300 python scripts/bench_overlap.py
M=4096 B=2048 CTX=700 step overlap_c 300 python scripts/bench_overlap.py
