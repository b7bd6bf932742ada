#!/bin/bash
# Two-phase ping-pong K-loop with 4 + 4 DMAs per phase (PH 3): numerics, A/B, PMC.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pp3_tests 400 env MLOP_GEMM_PP_PHASES=3 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or grouped or rope"
step pp3_ab 300 python -u scripts/bench_bigm.py
PMC1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
step pmc_pp3 120 env MLOP_GEMM_PP_PHASES=3 SHAPE=4096,4096,4096 BACKEND=mlop BIG_VARIANT=3 ITERS=10 rocprofv3 --pmc $PMC1 --kernel-trace --stats -d gpurun_out/r3pmc_pp3ph -o pmc -- python3 scripts/gemm_one.py
