#!/bin/bash
# EP = 2 Mixtral on one GPU: the EP GPU tests, then the control plane A/B (shm all-gather vs
# gloo) of the rehearsal bench, then a per-rank kernel trace of the shm tree for the idle-gap
# analysis (scripts/trace_window.py --by-pid)
B="python3 bench.py --gpus 2 --ep 2 --share-gpu --model mixtral-8x7b --batch 256 --steps 30 --warmup 5 --kv-gb 40 --no-operator"
bash scripts/steps.sh \
  "eptests 600 python -u -m pytest tests/test_ep_ipc_gpu.py tests/test_pod_multirank_gpu.py -x -v --timeout 300 --timeout-method thread" \
  "ep_shm1 400 $B" \
  "ep_gloo1 400 env MLOP_EP_CONTROL=gloo $B" \
  "ep_shm2 400 $B" \
  "ep_gloo2 400 env MLOP_EP_CONTROL=gloo $B" \
  "eptrace 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_ep2 -o ep_%pid% -- $B" \
  "epwin 120 sh -c 'python scripts/trace_window.py \$(find gpurun_out/prof_ep2 -name \"*kernel_trace.csv\") --by-pid --steps 20 --top 25'"
