#!/bin/bash
# Round-3 closing evidence, call A: the GPU suite, smoke, the default bench line and the
# driver's command at HEAD.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
step tests_r03f 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/tests_r03f.log
step smoke_r03f 200 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench_r03f 420 python3 -u bench.py
step driver_r03f 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
echo done
