#!/bin/bash
# Follow-up of run118: fewer, larger prompt batches per mixed step (prefill_min_batch 8 / 12,
# token budget 8192 / 10240), interleaved with the default.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step e_d1 300 python bench.py --no-operator
step e_pmb8 300 python bench.py --no-operator --prefill-min-batch 8
step e_pmb12 300 python bench.py --no-operator --prefill-min-batch 12
step e_d2 300 python bench.py --no-operator
step e_pmb8b 300 python bench.py --no-operator --prefill-min-batch 8
step e_pmb8_10k 300 python bench.py --no-operator --prefill-min-batch 8 --max-batched-tokens 10240
step e_pmb12_10k 300 python bench.py --no-operator --prefill-min-batch 12 --max-batched-tokens 10240
step e_d3 300 python bench.py --no-operator
