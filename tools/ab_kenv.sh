#!/bin/bash
# A/B an environment switch on the C2 step via tools/kernel_ab.py: bash tools/ab_kenv.sh VAR a b ...
VAR=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    env "$VAR=$v" timeout -k 10 120 python -u tools/kernel_ab.py --tag "$VAR=$v#$rep" 2>&1 | grep '^{' || exit 1
  done
done
