#!/bin/bash
# Round-3: launch tapes for the reference call pattern: drop-in tests, tape parity, dropin leg.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || { tail -40 "gpurun_out/$name.log"; exit $rc; }; }
summ() { python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/$1.log') if l.startswith('{')][-1]; print('$1', d['ms_per_step'], 'dropin', d['dropin_train']['ms_per_step'], d['dropin_train']['with_loss_item']['ms_per_step'])"; }
step r3m_dropin_tests 600 python3 -u -m pytest tests/test_gpu_dropin.py -x -v --timeout 200 --timeout-method thread
tail -3 gpurun_out/r3m_dropin_tests.log
step r3m_dropin_host 300 python3 -u tools/dropin_host.py --warmup 150 --steps 100
grep -v amdgpu.ids gpurun_out/r3m_dropin_host.log | head -60
B="python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-score --no-c4"
step r3m_bench 400 $B && summ r3m_bench
NCF_TAPE=0 step r3m_bench_notape 400 $B && summ r3m_bench_notape
step r3m_tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/r3m_tests.log
