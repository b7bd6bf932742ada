#!/bin/bash
# Hand-written GEMMs by default: GPU suite, smoke, headline bench (default and the auto/table
# A/B reference), small-batch decode both ways.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_def 600 python -u bench.py
step bench_auto 600 env MLOP_GEMM_BACKEND=auto python -u bench.py
step b64_def 300 python -u bench.py --batch 64 --steps 100 --warmup 20 --no-operator
step b64_auto 300 env MLOP_GEMM_BACKEND=auto python -u bench.py --batch 64 --steps 100 --warmup 20 --no-operator
step b16_def 300 python -u bench.py --batch 16 --steps 100 --warmup 20 --no-operator
step b16_auto 300 env MLOP_GEMM_BACKEND=auto python -u bench.py --batch 16 --steps 100 --warmup 20 --no-operator
