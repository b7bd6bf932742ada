#!/bin/bash
# Round 3: fixed GPU tests, HTTP-served bench, BASELINE configs 3 and 5 at real model size
# (controller/llm_demo.py: operator + real predictor processes on the GPU + canary gate).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step fixed_tests 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tp_gpu.py tests/test_kernels_gpu.py -k "tp2 or sample or mid_m" 
step ktime_test 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_model_gpu.py -k kernel_time
step bench_http 900 python -u bench.py --http --steps 40 --warmup 10
step demo_8b_promote 600 python -u -m mlopamd.controller.llm_demo --arch llama3-8b --concurrency 16 --timeout 500
step demo_8b_latency 600 python -u -m mlopamd.controller.llm_demo --arch llama3-8b --regress latency --concurrency 16 --timeout 500
step demo_mixtral_errors 900 python -u -m mlopamd.controller.llm_demo --arch mixtral-8x7b --regress errors --concurrency 16 --timeout 800
