#!/bin/bash
# flash prefill V fragments: read just in time (default) vs one 16-dim block ahead
# (MLOP_FLASH_VPIPE=1), interleaved on one box
bash scripts/steps.sh \
  "fa1 120 python3 scripts/bench_flash.py" "fp1 120 env MLOP_FLASH_VPIPE=1 python3 scripts/bench_flash.py" \
  "fa2 120 python3 scripts/bench_flash.py" "fp2 120 env MLOP_FLASH_VPIPE=1 python3 scripts/bench_flash.py" \
  "fa3 120 env S=1 L=8192 python3 scripts/bench_flash.py" "fp3 120 env S=1 L=8192 MLOP_FLASH_VPIPE=1 python3 scripts/bench_flash.py" \
  "fa4 120 env S=1 L=8192 python3 scripts/bench_flash.py" "fp4 120 env S=1 L=8192 MLOP_FLASH_VPIPE=1 python3 scripts/bench_flash.py" \
  "flt 300 env MLOP_FLASH_VPIPE=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k flash"
