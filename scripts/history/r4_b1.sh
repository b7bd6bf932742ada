#!/bin/bash
# Round 4 batch-1 decode sweep (one box): GEMV add+norm epilogue on/off, attention partition
# length, GEMV K-split threshold.  bench.py --batch 1 --steps 100 --warmup 20 --no-operator.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --batch 1 --steps 100 --warmup 20 --no-operator --cr-ready-samples 0"
step b1_base 300 $B
step b1_addnorm 300 env MLOP_GEMV_ADDNORM=1 MLOP_GEMV_ADDNORM_TESTS=1 $B
step b1_part256 300 env MLOP_ATTN_MIN_PART=256 $B
step b1_part512 300 env MLOP_ATTN_MIN_PART=512 $B
step b1_kw0 300 env MLOP_GEMV_KW4_SETS=0 $B
step b1_kw4k 300 env MLOP_GEMV_KW4_SETS=4096 $B
step b1_base2 300 $B
