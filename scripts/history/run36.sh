#!/bin/bash
# Eager HF baseline vs our engine; batch-1 latency; Mixtral-8x7B and Llama-3-70B (TP=1) on one GPU.
source scripts/gpu_check.sh
step eager_hf_b256 400 python scripts/bench_eager_hf.py
B=64 step eager_hf_b64 300 python scripts/bench_eager_hf.py
step bench_b256 300 python bench.py --batch 256 --steps 100 --warmup 20
step bench_b64 300 python bench.py --batch 64 --steps 100 --warmup 20
step bench_b1 300 python bench.py --batch 1 --steps 200 --warmup 20
step bench_mixtral 400 python bench.py --model mixtral-8x7b --batch 512 --steps 60 --warmup 10
step bench_70b 500 python bench.py --model llama3-70b --batch 256 --steps 40 --warmup 10
step bench_70b_b1 300 python bench.py --model llama3-70b --batch 1 --steps 60 --warmup 10 --no-operator
