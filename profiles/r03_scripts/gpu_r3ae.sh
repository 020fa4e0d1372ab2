#!/bin/bash
# Round-3: drop-in host trims (one-call dense .grad assignment, lighter tape checks).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; }; }
step r3ae_tests 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/r3ae_tests.log
B="python3 -u bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-score --no-c4"
for rep in 1 2 3; do
step r3ae_new_$rep 300 $B && python3 tools/bench_summ.py gpurun_out/r3ae_new_$rep.log
NCF_GRAD_SET=0 step r3ae_old_$rep 300 $B && python3 tools/bench_summ.py gpurun_out/r3ae_old_$rep.log
done
step r3ae_host 300 python3 -u tools/dropin_host.py --warmup 150 --steps 100
grep -v amdgpu.ids gpurun_out/r3ae_host.log | head -1
