#!/bin/bash
# Round-3 baseline: GEMM-only A/B at the headline row counts, PMC of the ping-pong kernel vs
# hipBLASLt (o and qkv shapes), then the default bench.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step gemm_ab 300 env BENCH_MS=2048,4088,4096 python -u scripts/bench_gemm.py
PMC1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for sh in 4096,4096,4096 4088,6144,4096; do
  for be in mlop hipblaslt; do
    tag=$(echo $sh | tr , x)_$be
    step pmc_$tag 120 env SHAPE=$sh BACKEND=$be ITERS=10 rocprofv3 --pmc $PMC1 --kernel-trace --stats -d gpurun_out/r3pmc_$tag -o pmc -- python3 scripts/gemm_one.py
  done
done
step bench 500 python bench.py --steps 20 --warmup 5
