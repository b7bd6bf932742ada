#!/bin/bash
source scripts/gpu_check.sh
step attn_decode 300 python scripts/bench_decode_attn.py
python scripts/smi_monitor.py gpurun_out/smi.jsonl > gpurun_out/smi_err.log 2>&1 &
MON=$!
step bench_default 600 python bench.py --steps 200 --warmup 20
kill $MON
