#!/bin/bash
# Confirm run119's best scheduler setting (prefill_min_batch 8 + a 10240-token step budget)
# against the default, interleaved, plus neighbours.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step f_d1 300 python bench.py --no-operator
step f_p8t10 300 python bench.py --no-operator --prefill-min-batch 8 --max-batched-tokens 10240
step f_p6t10 300 python bench.py --no-operator --prefill-min-batch 6 --max-batched-tokens 10240
step f_d2 300 python bench.py --no-operator
step f_p8t10b 300 python bench.py --no-operator --prefill-min-batch 8 --max-batched-tokens 10240
step f_p8t12 300 python bench.py --no-operator --prefill-min-batch 8 --max-batched-tokens 12288
step f_p4t10 300 python bench.py --no-operator --max-batched-tokens 10240
step f_d3 300 python bench.py --no-operator
step f_p8t10c 300 python bench.py --no-operator --prefill-min-batch 8 --max-batched-tokens 10240
