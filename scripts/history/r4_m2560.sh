#!/bin/bash
# the mixed steps' narrow GEMMs at ~2560 rows (160 tiles of 256x256 for o / down): default plan vs
# the ping-pong / four-wave kernels admitted from 128 tiles
G="python3 scripts/bench_gemm.py"
bash scripts/steps.sh \
  "m25d 600 env BENCH_MS=2560,3072 BENCH_TAG=d $G" \
  "m25p 600 env BENCH_MS=2560,3072 MLOP_GEMM_PP_MIN_TILES=128 BENCH_TAG=pp128 $G" \
  "m25w 600 env BENCH_MS=2560,3072 MLOP_GEMM_W4_MIN_TILES=128 BENCH_TAG=w4_128 $G"
