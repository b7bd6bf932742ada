#!/bin/bash
# decode attention V images double-buffered (default) vs single (MLOP_ATTN_VDB=0), same box,
# interleaved; attention tests in both modes
bash scripts/steps.sh \
  "kt_db 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k attention" \
  "kt_sb 600 env MLOP_ATTN_VDB=0 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k attention" \
  "db1 300 python3 scripts/bench_decode_attn.py" \
  "sb1 300 env MLOP_ATTN_VDB=0 python3 scripts/bench_decode_attn.py" \
  "db2 300 python3 scripts/bench_decode_attn.py" \
  "sb2 300 env MLOP_ATTN_VDB=0 python3 scripts/bench_decode_attn.py" \
  "startup 300 python3 scripts/probe_startup.py"
