#!/bin/bash
# Ping-pong GEMM with one half-tile of LDS-DMA per phase: numerics, A/B vs hipBLASLt, PMC,
# then the headline bench three ways: shipped table / re-tuned (table off) / all hand-written.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step gemm_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or grouped or rope"
step gemm_ab 300 python -u scripts/bench_bigm.py
PMC1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
step pmc_pp 120 env SHAPE=4096,4096,4096 BACKEND=mlop BIG_VARIANT=3 ITERS=10 rocprofv3 --pmc $PMC1 --kernel-trace --stats -d gpurun_out/r3pmc_pp3 -o pmc -- python3 scripts/gemm_one.py
step bench_table 600 python -u bench.py
step bench_retune 600 env MLOP_GEMM_TABLE=off python -u bench.py --save-gemm-table gpurun_out/gemm_table_r3.json
step bench_allmlop 600 env MLOP_GEMM_BACKEND=mlop python -u bench.py
