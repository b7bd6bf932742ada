#!/bin/bash
# Four-wave GEMM as the default large-M kernel: numerics + races, PMC at 4096^3, default bench.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step w4tests 300 python -u -m pytest tests/test_gemm_w4_gpu.py tests/test_races_gpu.py -x -q --timeout 120 --timeout-method thread
PMC1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
step pmc_w4 120 env SHAPE=4096,4096,4096 BACKEND=mlop BIG_VARIANT=5 ITERS=10 rocprofv3 --pmc $PMC1 --kernel-trace --stats -d gpurun_out/r3pmc_w4 -o pmc -- python3 scripts/gemm_one.py
step bench 600 python -u bench.py
