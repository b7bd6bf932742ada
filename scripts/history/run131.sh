#!/bin/bash
# Row-fitted small-M LDS-DMA tiles (gemm_small_tile 32 / 64): numerics, op-level A/B on cold
# rotating weights, end-to-end decode at batch 16 / 64 against the 64 x 64 tile (fresh autotune).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step st_tests 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "small_tiles or test_gemm_add_rmsnorm or test_gemm_silu"
step st_bench 300 env WSG_MIN_WG= SMALL_TILES=32,64 BENCH_MS=8,16,32,64 python scripts/bench_wsg.py
for b in 16 64; do
  for t in 0 32 64; do
    step e2e_st${t}_$b 200 env MLOP_GEMM_TABLE=off MLOP_GEMM_SMALL_TILE=$t python bench.py --batch $b --steps 100 --warmup 20 --no-operator
  done
done
