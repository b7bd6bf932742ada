#!/bin/bash
# Scheduler knobs at the headline config: how often prompts join the step (prefill_min_batch,
# max_decode_gap) and the per-step token budget; default runs interleaved for box drift.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step d1 300 python bench.py --no-operator
step pmb1 300 python bench.py --no-operator --prefill-min-batch 1
step pmb2 300 python bench.py --no-operator --prefill-min-batch 2
step d2 300 python bench.py --no-operator
step pmb8 300 python bench.py --no-operator --prefill-min-batch 8
step tok6k 300 python bench.py --no-operator --max-batched-tokens 6144
step pmb1_tok6k 300 python bench.py --no-operator --prefill-min-batch 1 --max-batched-tokens 6144
step d3 300 python bench.py --no-operator
