#!/bin/bash
# Round-3: deferred-Adam replay of a table pair as packed fp32 (adam0x2) vs scalar.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; }; }
summ() { python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/$1.log') if l.startswith('{')][-1]; k=d['kernel_ms_per_step']; print('$1', d['ms_per_step'], 'mlp_bwd', k.get('ncf_mlp_bwd'), 'sweep', k.get('ncf_adam_pairs_sweep_rolling'), 'catchup', k.get('ncf_adam_pairs_catchup_clock'), 'apply', k.get('ncf_adam_pairs_apply_clock'), 'iso', d['roofline']['isolated']['ms_per_launch'])"; }
step r3v_tests 600 python3 -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_parity.py -k "deferred or dense or hooked or bf16 or catchup or sweep or tapes" -x -q --timeout 200 --timeout-method thread
tail -2 gpurun_out/r3v_tests.log
step r3v_bf16 300 python3 -u -m pytest tests/test_gpu_bf16.py -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/r3v_bf16.log
B="python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-score --no-c4 --no-dropin"
for rep in 1 2; do
  step r3v_pk_$rep 300 $B && summ r3v_pk_$rep
  NCF_HIP_LIB=abl/lib_p0.so step r3v_p0_$rep 300 $B && summ r3v_p0_$rep
done
