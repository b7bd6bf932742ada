#!/bin/bash
# K7 PMC passes, both flash variants at 1 x 8192 (one rocprofv3 pass per counter set)
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES SQ_WAVE_CYCLES"
step pmc1 120 env S=1 L=8192 ITERS=3 rocprofv3 --pmc $P1 --kernel-trace -d gpurun_out/pmc_flash1 -o pmc -- python3 scripts/bench_flash.py
step pmc1_sum 60 python3 scripts/pmc_summary.py $(find gpurun_out/pmc_flash1 -name "*.db")
step pmc2 120 env S=1 L=8192 ITERS=3 rocprofv3 --pmc $P2 --kernel-trace -d gpurun_out/pmc_flash2 -o pmc -- python3 scripts/bench_flash.py
step pmc2_sum 60 python3 scripts/pmc_summary.py $(find gpurun_out/pmc_flash2 -name "*.db")
