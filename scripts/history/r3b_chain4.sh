#!/bin/bash
# Norm chain v3 (row totals by the producer band's last tile, consumer loads them by hidden
# LDS-DMA before the K-loop): numerics, kernel microbench, same-box windows, 100-step A/B.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step t_chain4 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_norm_chain_gpu.py tests/test_gemm_w4_gpu.py
step bench_chain4 300 python -u scripts/bench_chain.py
P="python3 bench.py --steps 40 --warmup 10 --no-operator"
step prof_on4 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_on4 -o bench --output-format csv -- $P
step win_on4 120 python scripts/trace_window.py gpurun_out/prof_on4/bench_kernel_trace.csv --steps 40 --top 30
rm -f gpurun_out/prof_on4/bench_kernel_trace.csv
export MLOP_NORM_CHAIN=0
step prof_off4 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_off4 -o bench --output-format csv -- $P
step win_off4 120 python scripts/trace_window.py gpurun_out/prof_off4/bench_kernel_trace.csv --steps 40 --top 30
rm -f gpurun_out/prof_off4/bench_kernel_trace.csv
unset MLOP_NORM_CHAIN
B="python3 bench.py --gpus 1 --steps 100 --warmup 10"
for i in 1 2; do
  step ab4_on_$i 400 $B
  step ab4_off_$i 400 env MLOP_NORM_CHAIN=0 $B
done
