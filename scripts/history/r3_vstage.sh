#!/bin/bash
# Two-phase ping-pong K-loop (now the only one) + V staged token-major in the fused QKV+RoPE
# epilogue: numerics, op-level A/B (V staging on / off), then the headline bench (shipped
# table / all hand-written).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step vs_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or grouped or rope"
step vs_bigm 300 python -u scripts/bench_bigm.py
step qkv_stage 200 env BENCH_MS=1024,2048,4088,8192 python -u scripts/bench_qkv_rope.py
step qkv_nostage 200 env MLOP_V_STAGE=0 BENCH_MS=1024,2048,4088,8192 python -u scripts/bench_qkv_rope.py
step bench_table 600 python -u bench.py
step bench_retune 600 env MLOP_GEMM_TABLE=off python -u bench.py --save-gemm-table gpurun_out/gemm_table_vs.json
step bench_allmlop 600 env MLOP_GEMM_BACKEND=mlop python -u bench.py
