#!/bin/bash
# Where does KV start-up time go right after another large GPU process on the same box?
# (first: a 200 GB allocate+touch process; then the default bench's deploy path, twice)
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step hog 120 python -c "
import torch,time
x=torch.empty(200*2**30,dtype=torch.uint8,device='cuda'); x.fill_(1); torch.cuda.synchronize(); print('hog done')"
step bench_after_hog 300 python bench.py --steps 5 --warmup 2
step bench_again 300 python bench.py --steps 5 --warmup 2
