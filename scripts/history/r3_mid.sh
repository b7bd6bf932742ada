#!/bin/bash
# Round-3 mid-round check: GEMM A/B (DMA split), pp PMC, GPU tests, smoke, bench, HTTP bench.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step gemm_ab 300 python -u scripts/bench_bigm.py
PMC1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
step pmc_pp 120 env SHAPE=4096,4096,4096 BACKEND=mlop BIG_VARIANT=3 ITERS=10 rocprofv3 --pmc $PMC1 --kernel-trace --stats -d gpurun_out/r3pmc_pp2 -o pmc -- python3 scripts/gemm_one.py
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python -u bench.py
step bench_http 900 python -u bench.py --http --steps 20 --warmup 5
