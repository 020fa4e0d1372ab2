#!/bin/bash
# Round-3: tower staging batches (NCF_STAGE_BATCH builds 1 / 5 (default) / 10), tower stamps, suite.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || { tail -40 "gpurun_out/$name.log"; exit $rc; }; }
summ() { python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/$1.log') if l.startswith('{')][-1]; k=d['kernel_ms_per_step']; print('$1', d['ms_per_step'], 'mlp', k.get('ncf_mlp_fwd'), k.get('ncf_mlp_bwd'), 'frac', d['roofline']['frac'], 'iso', d['roofline']['isolated']['ms_per_launch'], 'dropin', d['dropin_train']['ms_per_step'])"; }
step r3l_tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/r3l_tests.log
NCF_HIP_LIB=abl/lib_mstamps.so step r3l_mstamps 200 python3 -u tools/mlp_stamps.py
grep -v amdgpu.ids gpurun_out/r3l_mstamps.log
B="python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-score --no-c4"
step r3l_sb5 400 $B && summ r3l_sb5
NCF_HIP_LIB=abl/lib_sb1.so step r3l_sb1 400 $B && summ r3l_sb1
NCF_HIP_LIB=abl/lib_sb10.so step r3l_sb10 400 $B && summ r3l_sb10
step r3l_dropin_host 300 python3 -u tools/dropin_host.py --warmup 150 --steps 100
grep -v amdgpu.ids gpurun_out/r3l_dropin_host.log | head -100
