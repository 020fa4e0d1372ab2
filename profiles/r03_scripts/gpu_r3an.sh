#!/bin/bash
# Round-3: where the C5 item index build spends its time.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -30 "gpurun_out/$name.log"; exit $rc; }; }
step r3an_t 200 python3 -u tools/score_bench.py --reps 1 --k 10
grep -v amdgpu gpurun_out/r3an_t.log | head -5
step r3an_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3an_prof -o run --output-format csv -- python3 tools/score_bench.py --reps 1 --k 10
f=$(find gpurun_out/r3an_prof -name '*kernel_stats.csv' | head -1)
head -25 "$f" | cut -d, -f1-5
