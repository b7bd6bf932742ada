#!/bin/bash
# Four-wave GEMM body: numerics, then A/B vs the ping-pong kernel and hipBLASLt, then PMC.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step w4_tests 300 python -u -m pytest tests/test_gemm4w_gpu.py -x -v --timeout 120 --timeout-method thread
step w4_bench 300 python -u scripts/bench_gemm4w.py
PMC1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
step pmc_w4 120 env SHAPE=4096,4096,4096 BACKEND=mlop BIG_VARIANT=4 ITERS=10 rocprofv3 --pmc $PMC1 --kernel-trace --stats -d gpurun_out/r3pmc_w4 -o pmc -- python3 scripts/gemm_one.py
