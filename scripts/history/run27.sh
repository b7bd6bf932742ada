#!/bin/bash
# Fused QKV+RoPE epilogue: numerics, timing vs hipBLASLt + rope_cache, then the bench.
source scripts/gpu_check.sh
step pytest_rope 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "rope or gemm"
step bench_qkv_rope 300 python scripts/bench_qkv_rope.py
step bench_default 600 python bench.py --steps 100 --warmup 20
