#!/bin/bash
# Race screens: stream-K / grouped stream-K / fused split-KV tickets under a competing
# stream, and the host-sanitizer (TSan, ASan+UBSan) builds of the KV-arena harness.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step races 600 python -u -m pytest tests/test_races_gpu.py tests/test_native_sanitizers_gpu.py -v --timeout 200 --timeout-method thread
