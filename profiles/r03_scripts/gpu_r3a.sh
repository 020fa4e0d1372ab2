#!/bin/bash
# Round-3 first GPU pass: the driver's exact bench command, the drop-in probe (per-step times),
# and a kernel trace of the drop-in probe.  Every GPU step under its own limit; stop at the
# first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
step r3a_bench_driver 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-c4
tail -c 3000 gpurun_out/r3a_bench_driver.log
step r3a_dropin_probe 300 python3 -u tools/dropin_probe.py
cat gpurun_out/r3a_dropin_probe.log | tail -3
step r3a_dropin_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3a_dropin_prof -o run --output-format csv -- python3 tools/dropin_probe.py --trace 10 --windows 2
echo done
