#!/bin/bash
# Round-3: drop-in phases as hipGraphs vs launch tapes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -60 "gpurun_out/$name.log"; exit $rc; }; }
step r3ag_dropin_tests 600 python3 -u -m pytest tests/test_gpu_dropin.py -x -v --timeout 200 --timeout-method thread
tail -3 gpurun_out/r3ag_dropin_tests.log
step r3ag_tests 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/r3ag_tests.log
B="python3 -u bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-score --no-c4"
for rep in 1 2 3; do
step r3ag_graph_$rep 300 $B && python3 tools/bench_summ.py gpurun_out/r3ag_graph_$rep.log
NCF_DROPIN_GRAPH=0 step r3ag_tape_$rep 300 $B && python3 tools/bench_summ.py gpurun_out/r3ag_tape_$rep.log
done
step r3ag_host 300 python3 -u tools/dropin_host.py --warmup 150 --steps 100
grep -v amdgpu.ids gpurun_out/r3ag_host.log | head -1
