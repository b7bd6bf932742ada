#!/bin/bash
# PMC counters for the hand-written GEMM vs hipBLASLt on M=1024 / 8192 Llama shapes
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PMC1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES"
for sh in 8192,6144,4096 1024,6144,4096; do
  for be in mlop hipblaslt; do
    export SHAPE=$sh BACKEND=$be ITERS=10
    tag=$(echo $sh | tr , x)_$be
    step pmc_$tag 300 rocprofv3 --pmc $PMC1 --kernel-trace --stats -d gpurun_out/pmc_$tag -o pmc -- python3 scripts/gemm_one.py
  done
done
