#!/bin/bash
# M <= 128 GEMM tiles with a 6 / 5-stage LDS-DMA ring: numerics, then Llama batch 64 / 256
# A/B (stages 3 vs deep), alternating on one box.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_deep 300 env MLOP_GEMM_SMALL_STAGES=6 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "test_gemm or gemv or grouped or moe"
step b64_deep 600 env MLOP_GEMM_SMALL_STAGES=6 python bench.py --batch 64 --steps 100 --warmup 20 --no-operator
step b64_3 600 python bench.py --batch 64 --steps 100 --warmup 20 --no-operator
step b64_deep2 600 env MLOP_GEMM_SMALL_STAGES=6 python bench.py --batch 64 --steps 100 --warmup 20 --no-operator
step b64_32 600 python bench.py --batch 64 --steps 100 --warmup 20 --no-operator
step b256_deep 600 env MLOP_GEMM_SMALL_STAGES=6 python bench.py --batch 256 --steps 100 --warmup 20 --no-operator
step b256_3 600 python bench.py --batch 256 --steps 100 --warmup 20 --no-operator
