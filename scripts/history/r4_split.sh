#!/bin/bash
# mid-batch decode: split-K target of the small-M GEMMs (default 256 workgroups) vs 512 / 1024,
# batch 64 and 16, interleaved on one box
B="python3 bench.py --steps 100 --warmup 20 --no-operator --cr-ready-samples 0"
bash scripts/steps.sh \
  "s64_d 300 $B --batch 64" "s64_512 300 env MLOP_GEMM_SPLIT_TARGET=512 $B --batch 64" "s64_1k 300 env MLOP_GEMM_SPLIT_TARGET=1024 $B --batch 64" \
  "s16_d 300 $B --batch 16" "s16_512 300 env MLOP_GEMM_SPLIT_TARGET=512 $B --batch 16" "s16_1k 300 env MLOP_GEMM_SPLIT_TARGET=1024 $B --batch 16" \
  "s64_d2 300 $B --batch 64" "s64_512b 300 env MLOP_GEMM_SPLIT_TARGET=512 $B --batch 64"
