#!/bin/bash
# A/B the overlapped rolling sweep's fork/join points on the C2 step (tools/kernel_ab.py):
#   bash tools/ab_sweep.sh off "mlp_bwd:apply" "tower,mlp_bwd:apply" ...   (2 rounds)
# (fork points before the colon, comma-separated: one part of the slice per point)
for rep in 1 2; do
  for cfg in "$@"; do
    if [ "$cfg" = off ]; then
      NCF_OVERLAP_SWEEP=0 timeout -k 10 120 python -u tools/kernel_ab.py --tag "off#$rep" 2>&1 | grep '^{' || exit 1
    else
      NCF_OVERLAP_SWEEP=1 NCF_SWEEP_FORK=${cfg%%:*} NCF_SWEEP_JOIN=${cfg##*:} \
        timeout -k 10 120 python -u tools/kernel_ab.py --tag "$cfg#$rep" 2>&1 | grep '^{' || exit 1
    fi
  done
done
