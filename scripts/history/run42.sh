#!/bin/bash
# CU-partitioned attention / GEMM pipeline feasibility (scripts/bench_overlap.py, ATTN_CUS).
source scripts/gpu_check.sh
ATTN_CUS=32 step overlap_cu32 180 python scripts/bench_overlap.py
ATTN_CUS=64 step overlap_cu64 180 python scripts/bench_overlap.py
ATTN_CUS=48 step overlap_cu48 180 python scripts/bench_overlap.py
