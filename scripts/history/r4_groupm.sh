#!/bin/bash
# headline: the four-wave GEMM's grouped tile order (MLOP_GEMM_PP_GROUP_M, default 4) vs 2 / 8
H="python3 bench.py --no-operator --cr-ready-samples 0"
bash scripts/steps.sh \
  "g4a 600 $H" "g2a 600 env MLOP_GEMM_PP_GROUP_M=2 $H" "g8a 600 env MLOP_GEMM_PP_GROUP_M=8 $H" \
  "g4b 600 $H" "g2b 600 env MLOP_GEMM_PP_GROUP_M=2 $H" "g8b 600 env MLOP_GEMM_PP_GROUP_M=8 $H"
