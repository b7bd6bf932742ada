#!/bin/bash
# Residual add + RMSNorm fused into the decode GEMVs: all GPU tests, batch 1/2/4 decode, profile.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench_b1 300 python bench.py --batch 1 --steps 200 --warmup 20 --no-operator
step bench_b2 300 python bench.py --batch 2 --steps 200 --warmup 20 --no-operator
step bench_b4 300 python bench.py --batch 4 --steps 200 --warmup 20 --no-operator
step prof_b1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b1n -o b --output-format csv -- python3 bench.py --batch 1 --steps 100 --warmup 10 --no-operator
step bench_70b_b1 300 python bench.py --model llama3-70b --batch 1 --steps 60 --warmup 10 --no-operator
step bench_mixtral_b1 300 python bench.py --model mixtral-8x7b --batch 1 --steps 100 --warmup 10 --no-operator
