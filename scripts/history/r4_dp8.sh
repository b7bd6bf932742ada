#!/bin/bash
# the driver's SCALE path rehearsed on one GPU: bench.py --gpus 8 (self-launched DP ranks) and the
# torch.distributed.run form the driver uses, 8 DP replicas sharing cuda:0 (gloo; a functional
# check of launch, timing and aggregation, not a scaling number)
B="--share-gpu --batch 64 --steps 10 --warmup 3 --kv-gb 4 --no-operator --cr-ready-samples 0"
bash scripts/steps.sh \
  "dp8 500 python3 bench.py --gpus 8 $B" \
  "dp4run 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 $B"
