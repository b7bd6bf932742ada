#!/bin/bash
# batch 8-64 decode (split-K add + RMSNorm reduce with every load in flight), then the headline
# window of the final kernels (per-step kernel breakdown)
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step norm_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "norm or splitk or add_rms"
for b in 16 64; do
  step "b$b" 300 python3 bench.py --no-operator --batch $b --steps 60 --warmup 10 --cr-ready-samples 0
done
step prof64 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b64b -o b64 --output-format csv -- python3 bench.py --no-operator --batch 64 --steps 30 --warmup 5 --cr-ready-samples 0
step win64 120 python scripts/trace_window.py gpurun_out/prof_b64b/b64_kernel_trace.csv --steps 30 --top 25
rm -f gpurun_out/prof_b64b/b64_kernel_trace.csv
bash scripts/window.sh r5head 20
