#!/bin/bash
# Round-3: sweep fork before vs right after the tower backward launch (dispatch order).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; }; }
summ() { python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/$1.log') if l.startswith('{')][-1]; k=d['kernel_ms_per_step']; print('$1', d['ms_per_step'], 'mlp_bwd', k.get('ncf_mlp_bwd'), 'sweep', k.get('ncf_adam_pairs_sweep_rolling'), 'dropin', d['dropin_train']['ms_per_step'])"; }
B="python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-score --no-c4"
for rep in 1 2; do
  step r3u_def_$rep 300 $B && summ r3u_def_$rep
  NCF_SWEEP_FORK=mlp_bwd_after step r3u_after_$rep 300 $B && summ r3u_after_$rep
done
