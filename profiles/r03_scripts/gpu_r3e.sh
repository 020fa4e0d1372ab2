#!/bin/bash
# Round-3: GPU suite, then the driver's bench command (drop-in / C4 legs with the claim catch-up
# and the fused D=128 kernels).  Each GPU step under its own limit; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || { tail -40 "gpurun_out/$name.log"; exit $rc; }; }
step r3e_tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
tail -2 gpurun_out/r3e_tests.log
step r3e_bench 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
tail -c 600 gpurun_out/r3e_bench.log
