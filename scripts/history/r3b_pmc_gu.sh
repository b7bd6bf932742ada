#!/bin/bash
# Counters of gate_up at M = 4088 (the shape where the four-wave kernel trails hipBLASLt by 5 %):
# L2 hit/miss and HBM read requests, then the SQ stall picture, one counter pass per run.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TCC="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for be in mlop hipblaslt; do
  step tcc_$be 90 env SHAPE=4088,28672,4096 EPI=$([ $be = mlop ] && echo 1 || echo 0) BACKEND=$be ITERS=10 timeout -s KILL 80 rocprofv3 --pmc $TCC --kernel-trace -d gpurun_out/pmc_gu_tcc_$be -o pmc -- python3 scripts/gemm_one.py
  step sq_$be 90 env SHAPE=4088,28672,4096 EPI=$([ $be = mlop ] && echo 1 || echo 0) BACKEND=$be ITERS=10 timeout -s KILL 80 rocprofv3 --pmc $SQ --kernel-trace -d gpurun_out/pmc_gu_sq_$be -o pmc -- python3 scripts/gemm_one.py
  step fetch_$be 90 env SHAPE=4088,28672,4096 EPI=$([ $be = mlop ] && echo 1 || echo 0) BACKEND=$be ITERS=10 timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_gu_fetch_$be -o pmc -- python3 scripts/gemm_one.py
done
