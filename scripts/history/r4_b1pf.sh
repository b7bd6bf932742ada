#!/bin/bash
# GEMV QKV RoPE epilogue with its slot / position / cos-sin loads issued behind the weight stream:
# kernel tests, batch-1 bench twice, batch-1 kernel window
bash scripts/steps.sh \
  "kt 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_races_gpu.py" \
  "b1a 300 python3 bench.py --batch 1 --steps 100 --warmup 20 --no-operator --cr-ready-samples 0" \
  "b1b 300 python3 bench.py --batch 1 --steps 100 --warmup 20 --no-operator --cr-ready-samples 0" \
  "b1prof 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_b1pf -o b1 -- python3 bench.py --batch 1 --steps 40 --warmup 20 --no-operator --cr-ready-samples 0" \
  "b1win 60 python scripts/trace_window.py gpurun_out/prof_b1pf/b1_kernel_trace.csv --steps 20 --top 14"
