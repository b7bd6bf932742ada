#!/bin/bash
# where the predictor's start-up goes: python -X importtime of torch alone and of the server
# module's first-request imports (the ones the predictor makes before it is ready)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -X importtime -c "import torch" 2> gpurun_out/imp_torch.log
timeout -k 10 300 python3 -X importtime -c "import mlopamd.runtime.server, mlopamd.runtime.engine, mlopamd.models, mlopamd.ops" 2> gpurun_out/imp_server.log
timeout -k 10 300 python3 -c "
import time; t=time.perf_counter(); import torch; t1=time.perf_counter()
import mlopamd.runtime.server, mlopamd.runtime.engine, mlopamd.models, mlopamd.ops; t2=time.perf_counter()
print('torch', round(t1-t,3), 'ours', round(t2-t1,3))" > gpurun_out/imp_wall.log
