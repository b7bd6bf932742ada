#!/bin/bash
# batch-1 decode with the GEMV norm chain under counters: bytes fetched from HBM per kernel
# (FETCH_SIZE) and the busy clock (GRBM_GUI_ACTIVE), one rocprofv3 --pmc pass
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pmcb1 240 timeout -s KILL 220 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_b1 -o pmc -- \
  python3 bench.py --batch 1 --steps 10 --warmup 3 --no-operator --cr-ready-samples 0
step pmcb1sum 60 python3 scripts/pmc_summary.py gpurun_out/pmc_b1/pmc_results.db
