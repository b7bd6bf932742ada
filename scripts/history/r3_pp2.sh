#!/bin/bash
# Ping-pong GEMM, two-phase K-loop (2 x 32 MFMAs per K-tile, half the group hand-offs):
# numerics of every pp launch form under it, then A/B vs the 4-phase loop and hipBLASLt, PMC.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pp2_tests 400 env MLOP_GEMM_PP_PHASES=2 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or grouped or rope"
step pp2_ab 300 python -u scripts/bench_bigm.py
PMC1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
step pmc_pp2 120 env MLOP_GEMM_PP_PHASES=2 SHAPE=4096,4096,4096 BACKEND=mlop BIG_VARIANT=3 ITERS=10 rocprofv3 --pmc $PMC1 --kernel-trace --stats -d gpurun_out/r3pmc_pp2ph -o pmc -- python3 scripts/gemm_one.py
