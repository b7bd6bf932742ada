#!/bin/bash
# mixed prefill+decode steps: correctness on GPU, then bench policy variants
source scripts/gpu_check.sh
step pytest_mixed 600 python -m pytest tests/test_model_gpu.py -q -m gpu -x
step b_nomixed 600 python bench.py --steps 100 --warmup 40 --no-mixed
step b_mixed16 600 python bench.py --steps 100 --warmup 40
step b_mixed1 600 python bench.py --steps 100 --warmup 40 --prefill-min-batch 1 --max-decode-gap 0
step b_mixed4 600 python bench.py --steps 100 --warmup 40 --prefill-min-batch 4
