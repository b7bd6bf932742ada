#!/bin/bash
# round-end rehearsal on the final (non-temporal stream) tree: GPU suite, smoke(), the driver's
# command, the Llama batch sweep, Mixtral / 70B rows, long context
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step gpu_suite 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step driver 500 python3 bench.py --gpus 1 --steps 20 --warmup 5
for b in 1 4 16 64 256 512 1024 2048; do
  step "sw_b$b" 300 python3 bench.py --no-operator --batch $b --steps 40 --warmup 10 --cr-ready-samples 0
done
for b in 1 64 256 1024; do
  step "sw_mix$b" 400 python3 bench.py --no-operator --model mixtral-8x7b --batch $b --steps 30 --warmup 10 --cr-ready-samples 0
done
step sw_70b1 400 python3 bench.py --no-operator --model llama3-70b --batch 1 --steps 30 --warmup 5 --cr-ready-samples 0
step long32k 500 python3 bench.py --no-operator --model llama3.1-8b --batch 16 --prompt-len 32000 --output-len 256 --max-model-len 32768 --steps 100 --warmup 10 --cr-ready-samples 0
