#!/bin/bash
# single-buffer V images with page ids one pair ahead; predictor HIP warm-up thread (torch's own
# runtime): attention tests, decode-attention bench, start-up probe, the driver bench twice
bash scripts/steps.sh \
  "kt 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_races_gpu.py" \
  "dattn 300 python3 scripts/bench_decode_attn.py" \
  "startup 300 python3 scripts/probe_startup.py" \
  "bench_a 600 python3 bench.py --gpus 1 --steps 20 --warmup 5" \
  "bench_b 600 python3 bench.py --gpus 1 --steps 20 --warmup 5"
