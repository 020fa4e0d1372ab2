#!/bin/bash
# Round-3: tower backward head phase with all of a thread's row loads issued first.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; }; }
summ() { python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/$1.log') if l.startswith('{')][-1]; k=d['kernel_ms_per_step']; print('$1', d['ms_per_step'], 'mlp_bwd', k.get('ncf_mlp_bwd'), 'iso', d['roofline']['isolated']['ms_per_launch'], 'frac', d['roofline']['frac'])"; }
step r3y_tests 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/r3y_tests.log
B="python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-score --no-c4 --no-dropin"
for rep in 1 2; do
  step r3y_new_$rep 300 $B && summ r3y_new_$rep
  NCF_HIP_LIB=abl/lib_old.so step r3y_old_$rep 300 $B && summ r3y_old_$rep
done
