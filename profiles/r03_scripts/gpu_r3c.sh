#!/bin/bash
# Round-3: the GPU suite (new: 200-step parity, lr change under graph, engine-wide id flag) and
# the default bench line.  Each GPU step under its own limit; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || { tail -30 "gpurun_out/$name.log"; exit $rc; }; }
step r3c_new 300 python3 -u -m pytest tests/test_gpu_long.py tests/test_gpu_dropin.py tests/test_gpu_parity.py -k "200_step or survey_tol or rare_batch or reports_bad or lr_change or out_of_range or score" -x -v -s --timeout 200 --timeout-method thread
grep -E "parity:|dprob|passed|failed" gpurun_out/r3c_new.log | tail -8
step r3c_tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
tail -3 gpurun_out/r3c_tests.log
step r3c_bench 900 python3 -u bench.py --steps 20 --warmup 5
tail -c 1500 gpurun_out/r3c_bench.log
