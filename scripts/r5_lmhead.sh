#!/bin/bash
# lm_head GEMM (N = 128256) at the headline's logits row counts vs the library
source scripts/gpu_check.sh
step lmhead 300 python -u scripts/bench_mid_m.py --ms 1024,2040,2048 --shapes lm_head --iters 5
