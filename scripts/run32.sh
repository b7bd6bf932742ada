#!/bin/bash
# Full-size configs 4/5 models on ONE MI355X (both fit 288 GB): Mixtral-8x7B (93 GB, MoE grouped GEMM)
# and Llama-3-70B (141 GB, TP=1 here; TP=8 needs the 8-GPU node).
source scripts/gpu_check.sh
step bench_mixtral 600 python bench.py --model mixtral-8x7b --batch 512 --steps 60 --warmup 10
step bench_70b 600 python bench.py --model llama3-70b --batch 256 --steps 40 --warmup 5
