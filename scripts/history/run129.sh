#!/bin/bash
# End-to-end A/B of the GEMM backend choices at the headline's row counts (M buckets 2048 / 4096):
# shipped table vs t1 (fused SiLU-mul gate_up and fused RoPE QKV on the hand-written kernel) vs
# t2 (every projection on the hand-written kernel), interleaved on one box.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  step ab_t0_$r 300 python bench.py --steps 100 --warmup 20 --no-operator
  step ab_t1_$r 300 env MLOP_GEMM_TABLE=build/tables/t1.json python bench.py --steps 100 --warmup 20 --no-operator
  step ab_t2_$r 300 env MLOP_GEMM_TABLE=build/tables/t2.json python bench.py --steps 100 --warmup 20 --no-operator
done
