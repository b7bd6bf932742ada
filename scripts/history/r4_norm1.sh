#!/bin/bash
# batch-1 add+RMSNorm: norm weights loaded with the row (both kernel forms); block form (default
# below 256 rows) vs the wave form (MLOP_NORM_WAVE_MIN_M=1), interleaved on one box; flash prefill
# with the V fragments read one 16-dim block ahead
bash scripts/steps.sh \
  "nt 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k norm" \
  "blk1 300 python3 bench.py --batch 1 --steps 100 --warmup 20 --no-operator --cr-ready-samples 0" \
  "wav1 300 env MLOP_NORM_WAVE_MIN_M=1 python3 bench.py --batch 1 --steps 100 --warmup 20 --no-operator --cr-ready-samples 0" \
  "blk2 300 python3 bench.py --batch 1 --steps 100 --warmup 20 --no-operator --cr-ready-samples 0" \
  "wav2 300 env MLOP_NORM_WAVE_MIN_M=1 python3 bench.py --batch 1 --steps 100 --warmup 20 --no-operator --cr-ready-samples 0" \
  "b1prof 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_b1n -o b1 -- python3 bench.py --batch 1 --steps 40 --warmup 20 --no-operator --cr-ready-samples 0" \
  "b1win 60 python scripts/trace_window.py gpurun_out/prof_b1n/b1_kernel_trace.csv --steps 20 --top 12" \
  "fl1 120 python3 scripts/bench_flash.py" \
  "fl2 120 env S=1 L=8192 python3 scripts/bench_flash.py" \
  "flt 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k flash"
