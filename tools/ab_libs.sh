#!/bin/bash
# A/B library builds on the C2 step: bash tools/ab_libs.sh abl/a.so abl/b.so ...  (2 rounds)
for rep in 1 2; do
  for lib in "$@"; do
    NCF_HIP_LIB=$PWD/$lib timeout -k 10 120 python -u tools/kernel_ab.py --tag "$lib#$rep" $AB_ARGS 2>&1 | grep '^{' || exit 1
  done
done
