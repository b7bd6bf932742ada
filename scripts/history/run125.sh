#!/bin/bash
# wsgemm.hip (register-streamed MFMA GEMM for 4 < M <= 64): numerics, op-level A/B against the
# LDS-DMA tiles and hipBLASLt on rotating (cold) weights, then end-to-end decode at batch 16 / 64
# with wsgemm on vs off (fresh autotune in both arms).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step wsg_tests 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "wsg or gemv or gemm_add_rmsnorm or gemm_silu"
step wsg_bench 300 env WSG_MIN_WG=128,256,512 python scripts/bench_wsg.py
for b in 64 16; do
  step e2e_on_$b 200 env MLOP_GEMM_TABLE=off python bench.py --batch $b --steps 100 --warmup 20 --no-operator
  step e2e_off_$b 200 env MLOP_GEMM_TABLE=off MLOP_WSG_MAX_M=0 python bench.py --batch $b --steps 100 --warmup 20 --no-operator
done
