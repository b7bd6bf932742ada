#!/bin/bash
# Llama-3-70B projection shapes: hand-written GEMM vs hipBLASLt (torch.matmul) at M = 256 / 512 / 2048
bash scripts/steps.sh "g70 600 env BENCH_MODEL=70b BENCH_MS=256,512,2048 python3 scripts/bench_gemm.py"
