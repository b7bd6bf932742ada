#!/bin/bash
# NOTE: gemm4.hip (the four-wave kernel) was removed after this run: profiles/r02_gemm_fourwave_rejected.md
# PMC counters at M=4096 N=4096 K=14336 (down projection): ping-pong (3) vs four-wave (4) vs hipBLASLt.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PMC1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES"
export SHAPE=4096,4096,14336 ITERS=10
for v in 3 4 lib; do
  if [ $v = lib ]; then export BACKEND=hipblaslt; else export BACKEND=mlop BIG_VARIANT=$v; fi
  step pmc_v$v 120 rocprofv3 --pmc $PMC1 --kernel-trace --stats -d gpurun_out/pmc65_v$v -o pmc -- python3 scripts/gemm_one.py
done
