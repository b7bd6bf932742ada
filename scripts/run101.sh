#!/bin/bash
# K7 flash prefill restructured (K fragments read once for both column tiles, V read just in
# time per 16-dim block: 214 -> 168 VGPRs, 2 -> 3 waves per SIMD): numerics + microbench.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_flash 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash or paged_attention or attention"
step flash_4x2048 200 env CHECK=1 python scripts/bench_flash.py
step flash_1x8192 200 env S=1 L=8192 python scripts/bench_flash.py
step flash_16x512 200 env S=16 L=512 python scripts/bench_flash.py
