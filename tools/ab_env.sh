#!/bin/bash
# A/B an environment switch on the C2 bench: bash tools/ab_env.sh VAR val_a val_b
mkdir -p gpurun_out
VAR=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    env_line="$VAR=$v"
    export "$env_line"
    timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-score > gpurun_out/abe_${v}_$rep.log 2>&1 || exit $?
    python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/abe_${v}_$rep.log') if l.startswith('{')][-1])
print('$VAR=$v', $rep, d['ms_per_step'])"
  done
done
