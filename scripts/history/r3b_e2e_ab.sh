#!/bin/bash
# End-to-end A/B on one box (interleaved): async scheduling on/off, four-wave vs ping-pong GEMM;
# then the timed-window kernel profile of the default configuration.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python -u bench.py --steps 100 --warmup 30 --no-operator"
step bench_def_a 400 $B
step bench_sync_a 400 $B --no-async
step bench_v3_a 400 env MLOP_GEMM_BIG_VARIANT=3 $B
step bench_def_b 400 $B
step bench_sync_b 400 $B --no-async
step bench_v3_b 400 env MLOP_GEMM_BIG_VARIANT=3 $B
step prof_w4 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_w4 -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 10 --no-operator
step window_w4 120 python scripts/trace_window.py gpurun_out/prof_w4/bench_kernel_trace.csv --steps 20 --top 40
rm -f gpurun_out/prof_w4/bench_kernel_trace.csv.gz
