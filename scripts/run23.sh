#!/bin/bash
# Re-validate after container re-creation; re-measure GEMM choices with the ping-pong kernel.
source scripts/gpu_check.sh
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bg_pp3 400 env BENCH_MS=1024,1536,2048,3072,4096 BENCH_TAG=pp3 python scripts/bench_gemm.py
step bench_fresh 600 env MLOP_GEMM_TABLE=off python bench.py --steps 100 --warmup 40 --save-gemm-table gpurun_out/gemm_table_new.json
