#!/bin/bash
# MoE decode tilings (scripts/bench_moe_decode.py) and a Mixtral batch-64 window, after the EP
# control-plane run (scripts/r5_ep.sh)
bash scripts/r5_ep.sh && bash scripts/steps.sh \
  "moedec 600 python -u scripts/bench_moe_decode.py --rows 128,256,512,2048" \
  "prof_mix64 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mix64 -o bench --output-format csv -- python3 bench.py --model mixtral-8x7b --batch 64 --steps 20 --warmup 10 --no-operator --cr-ready-samples 0" \
  "win_mix64 120 python scripts/trace_window.py gpurun_out/prof_mix64/bench_kernel_trace.csv --steps 20 --top 30"
