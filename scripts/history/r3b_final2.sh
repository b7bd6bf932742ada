#!/bin/bash
# Final same-box numbers: driver command with four-wave vs ping-pong GEMMs (interleaved), then
# the timed-window kernel profile of the default.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --gpus 1 --steps 20 --warmup 5"
step d_v5a 400 $B
step d_v3a 400 env MLOP_GEMM_BIG_VARIANT=3 $B
step d_v5b 400 $B
step d_v3b 400 env MLOP_GEMM_BIG_VARIANT=3 $B
step prof_final 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 10 --no-operator
step window_final 120 python scripts/trace_window.py gpurun_out/prof_final/bench_kernel_trace.csv --steps 20 --top 40
rm -f gpurun_out/prof_final/bench_kernel_trace.csv.gz
