#!/bin/bash
# Ping-pong GEMM with buffer-form LDS-DMA issue: numerics, A/B, PMC, bench.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step bl_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or grouped or rope or moe"
step bl_ab 300 python -u scripts/bench_bigm.py
PMC1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
step pmc_bl 120 env SHAPE=4096,4096,4096 BACKEND=mlop BIG_VARIANT=3 ITERS=10 rocprofv3 --pmc $PMC1 --kernel-trace --stats -d gpurun_out/r3pmc_bl -o pmc -- python3 scripts/gemm_one.py
step bench_bl 600 env MLOP_GEMM_TABLE=off python -u bench.py --save-gemm-table gpurun_out/gemm_table_bl.json
step bench_bl_allmlop 600 env MLOP_GEMM_BACKEND=mlop python -u bench.py
