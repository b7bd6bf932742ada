#!/bin/bash
# Round 4 counters: the fused QKV projection (EPI 3: RoPE + paged K + V
# staging) vs the plain QKV GEMM vs gate_up (EPI 1) at M = 4088, four-wave kernel; one counter
# pass per run (rocprofv3 --pmc with --kernel-trace only).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
TCC="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
run() {  # name shape epi
  step "sq_$1" 90 env SHAPE=$2 EPI=$3 ITERS=10 timeout -s KILL 80 rocprofv3 --pmc $SQ --kernel-trace -d "gpurun_out/pmc_$1_sq" -o pmc -- python3 scripts/gemm_one.py
  step "tcc_$1" 90 env SHAPE=$2 EPI=$3 ITERS=10 timeout -s KILL 80 rocprofv3 --pmc $TCC --kernel-trace -d "gpurun_out/pmc_$1_tcc" -o pmc -- python3 scripts/gemm_one.py
}
run qkv_rope 4088,6144,4096 3
run qkv_plain 4088,6144,4096 0
run o_plain 4088,4096,4096 0
run gate_up 4088,28672,4096 1
step bigm 300 env BENCH_MS=4088 BENCH_VARIANTS=5 python3 scripts/bench_bigm.py
step ropevar 300 python3 scripts/bench_rope_var.py
