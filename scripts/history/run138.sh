#!/bin/bash
# Per-shape small-M tiles (BM 16: qkv/o/down BN 32 + 8-deep ring, gate_up BN 64 + 6-deep):
# numerics, op level, and batch 8 / 16 decode vs the previous default (BN 64, 4-deep).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step auto_tests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 150 --timeout-method thread -k "rope or engine or small_tiles"
step auto_bench 200 env WSG_MIN_WG= SMALL_TILES=1,64 BENCH_MS=8,16 python scripts/bench_wsg.py
for r in 1 2; do
  for b in 8 16; do
    step e2e_t64_${b}_$r 200 env MLOP_GEMM_SMALL_TILE=64 python bench.py --batch $b --steps 150 --warmup 20 --no-operator
    step e2e_auto_${b}_$r 200 python bench.py --batch $b --steps 150 --warmup 20 --no-operator
  done
done
