#!/bin/bash
# Planner sweeps: MoE grouped tilings over the decode routing range (including exact per-expert
# counts at the 256-row boundary), and the dense mid-M projections vs hipBLASLt
bash scripts/steps.sh \
  "moedec2 900 python -u scripts/bench_moe_decode.py --rows 384,512,768,1024,1536" \
  "moecnt 600 python -u scripts/bench_moe_decode.py --counts '256,256,256,256,256,256,256,256;257,257,257,257,257,257,257,257;250,250,250,250,250,250,250,250;272,272,272,272,240,240,240,240'" \
  "midm 1100 python -u scripts/bench_mid_m.py"
