#!/bin/bash
# Norm chain with the row factors computed before the K-loop: numerics, same-box window
# profiles on / off, then 100-step driver-style A/B pairs.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step t_chain2 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_norm_chain_gpu.py tests/test_gemm_w4_gpu.py
P="python3 bench.py --steps 40 --warmup 10 --no-operator"
step prof_on2 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_on2 -o bench --output-format csv -- $P
step win_on2 120 python scripts/trace_window.py gpurun_out/prof_on2/bench_kernel_trace.csv --steps 40 --top 30
rm -f gpurun_out/prof_on2/bench_kernel_trace.csv
export MLOP_NORM_CHAIN=0
step prof_off2 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_off2 -o bench --output-format csv -- $P
step win_off2 120 python scripts/trace_window.py gpurun_out/prof_off2/bench_kernel_trace.csv --steps 40 --top 30
rm -f gpurun_out/prof_off2/bench_kernel_trace.csv
unset MLOP_NORM_CHAIN
B="python3 bench.py --gpus 1 --steps 100 --warmup 10"
for i in 1 2; do
  step ab2_on_$i 400 $B
  step ab2_off_$i 400 env MLOP_NORM_CHAIN=0 $B
done
