#!/bin/bash
# Round-3: one fused C2 step's timeline per queue (critical path and idle gaps).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -30 "gpurun_out/$name.log"; exit $rc; }; }
step r3aq_prof 300 rocprofv3 --kernel-trace -d gpurun_out/r3aq_prof -o run --output-format csv -- python3 tools/kernel_ab.py --warmup 140 --steps 200
f=$(find gpurun_out/r3aq_prof -name '*kernel_trace.csv' | head -1)
python3 tools/step_timeline.py "$f" k_gather_ln_gmf 0.5 > gpurun_out/r3aq_timeline.txt
python3 tools/step_timeline.py "$f" k_gather_ln_gmf 0.6 > gpurun_out/r3aq_timeline2.txt
rm -f "$f"
cat gpurun_out/r3aq_timeline.txt
