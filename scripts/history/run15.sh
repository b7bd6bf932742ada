#!/bin/bash
# bench: default + larger concurrency; kernel profile of the default (mixed-step) bench
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_k 600 python -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -q -m gpu -x -k "argmax or flash or attention or engine or llama3"
step b_default 600 python bench.py --steps 100 --warmup 40
step b_1536 600 python bench.py --steps 100 --warmup 40 --batch 1536
step b_2048 600 python bench.py --steps 100 --warmup 40 --batch 2048
step prof_mixed 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o bench --output-format csv -- python3 bench.py --steps 60 --warmup 40 --no-operator
step pytest_canary 900 python -m pytest tests/test_llm_canary_gpu.py -q -m gpu -x
