#!/bin/bash
# per-shape timings of MLOP_GEMM_BACKEND=auto at batch 512 (which mixed-step GEMMs go to hipBLASLt)
bash scripts/steps.sh "ad 600 python3 scripts/history/dump_auto.py --batch 512 --steps 60 --warmup 10 --no-operator --cr-ready-samples 0"
