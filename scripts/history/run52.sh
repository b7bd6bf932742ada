#!/bin/bash
# Split-KV attention combined in-launch by the last-arriving partition: numerics, then
# small-batch decode with the in-launch combine vs the separate reduce launch.
source scripts/gpu_check.sh
cd "$GRAFT_REPO_ROOT"
step attn_tests 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "attention or flash" --timeout 120 --timeout-method thread
step b1_fused 300 python bench.py --batch 1 --steps 200 --warmup 20 --no-operator
MLOP_ATTN_FUSED_REDUCE=0 step b1_sep 300 python bench.py --batch 1 --steps 200 --warmup 20 --no-operator
step b8_fused 300 python bench.py --batch 8 --steps 200 --warmup 20 --no-operator
MLOP_ATTN_FUSED_REDUCE=0 step b8_sep 300 python bench.py --batch 8 --steps 200 --warmup 20 --no-operator
step b1_fused2 300 python bench.py --batch 1 --steps 200 --warmup 20 --no-operator
