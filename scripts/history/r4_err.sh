#!/bin/bash
# host-mapped error words of the IPC collectives (polled every engine step): the multi-process
# GPU tests (custom all-reduce incl. the contention screen, EP exchange, TP engine)
bash scripts/steps.sh \
  "mp 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_custom_ar_gpu.py tests/test_ep_ipc_gpu.py tests/test_tp_gpu.py"
