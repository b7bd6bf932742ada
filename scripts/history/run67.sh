#!/bin/bash
# Lazily backed KV arena (vmm.hip): GPU tests, then start-up after a 200 GB process (cf. run66.sh).
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_kv_lazy 300 python -u -m pytest tests/test_kv_lazy_gpu.py -x -v --timeout 120 --timeout-method thread
step hog 120 python -c "
import torch
x=torch.empty(200*2**30,dtype=torch.uint8,device='cuda'); x.fill_(1); torch.cuda.synchronize(); print('hog done')"
step bench_after_hog 300 python bench.py --steps 20 --warmup 5
step bench_default 400 python bench.py
