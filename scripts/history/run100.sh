#!/bin/bash
# K7 flash prefill: throughput at 4 x 2048 and 1 x 8192 causal prompts, then PMC counters.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step flash_4x2048 200 env CHECK=1 python scripts/bench_flash.py
step flash_1x8192 200 env S=1 L=8192 python scripts/bench_flash.py
step flash_16x512 200 env S=16 L=512 python scripts/bench_flash.py
PMC="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"
step flash_pmc 120 timeout -s KILL 100 rocprofv3 --pmc $PMC --kernel-trace --stats -d gpurun_out/pmc100 -o pmc -- python3 scripts/bench_flash.py
