#!/bin/bash
# PMC pass over the chain microbench: plain SiLU gate_up (<1>) vs row-scaled (<9>), O plain (<0>)
# vs residual add + sums of squares (<4>).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pmc_chain 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --stats -d gpurun_out/pmc_chain -o pmc --output-format csv -- python3 scripts/bench_chain.py
