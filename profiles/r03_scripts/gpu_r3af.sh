#!/bin/bash
# Round-3: whole-step hipGraph replay vs eager (GPU overhead of graph nodes today).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; }; }
B="python3 -u bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-score --no-c4 --no-dropin"
for rep in 1 2; do
step r3af_eager_$rep 300 $B && python3 tools/bench_summ.py gpurun_out/r3af_eager_$rep.log
step r3af_graph_$rep 300 $B --graph && python3 tools/bench_summ.py gpurun_out/r3af_graph_$rep.log
done
