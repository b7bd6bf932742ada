#!/bin/bash
# Llama-3-8B projection shapes at M = 256 / 512 / 1024: hand-written GEMM vs hipBLASLt
bash scripts/steps.sh "g8 600 env BENCH_MS=256,512,1024 python3 scripts/bench_gemm.py"
