#!/bin/bash
# Engine host-path trim: GPU engine tests, default bench (host us per step in step_mix), batch 1.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step engine_gpu 600 python -u -m pytest tests/test_model_gpu.py tests/test_tp_gpu.py tests/test_llm_canary_gpu.py -x -q --timeout 200 --timeout-method thread
step bench_default 400 python bench.py
step bench_b1 300 python bench.py --batch 1 --steps 300 --warmup 20 --no-operator
