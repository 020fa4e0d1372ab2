#!/bin/bash
# Round-3: tower backward LayerNorm backward row loads preloaded.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; }; }
summ() { python3 tools/bench_summ.py gpurun_out/$1.log ncf_mlp_bwd ncf_adam_pairs_apply_clock ncf_adam_pairs_catchup_clock; }
step r3z_tests 600 python3 -u -m pytest tests/test_gpu_parity.py -k "mlp or tower or train or golden" -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/r3z_tests.log
B="python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-score --no-c4 --no-dropin"
for rep in 1 2; do
  step r3z_new_$rep 300 $B && summ r3z_new_$rep
  NCF_HIP_LIB=abl/lib_old.so step r3z_old_$rep 300 $B && summ r3z_old_$rep
done
