#!/bin/bash
# A/B (rolling-sweep fork point, next-batch dedup fork point) pairs on the C2 step:
#   bash tools/ab_forks.sh mlp_bwd:attn_bwd tower:attn_bwd ...   (2 rounds)
for rep in 1 2; do
  for cfg in "$@"; do
    NCF_SWEEP_FORK=${cfg%%:*} NCF_DEDUP_FORK=${cfg##*:} \
      timeout -k 10 120 python -u tools/kernel_ab.py --tag "$cfg#$rep" 2>&1 | grep '^{' || exit 1
  done
done
