#!/bin/bash
# Round-3: stream-only events (scope 2 default) and the step-start event recorded only when the
# dedup forks there: GPU suite, interleaved fused-step A/B against scope 0, timeline.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; }; }
step r3aw_tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/r3aw_tests.log
for rep in 1 2 3; do
for sc in 0 2; do
NCF_EVENT_SCOPE=$sc step r3aw_ab_${sc}_$rep 200 python3 -u tools/kernel_ab.py --tag scope$sc
echo "scope $sc: fused $(grep '^{' gpurun_out/r3aw_ab_${sc}_$rep.log | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
done
done
step r3aw_tl 300 rocprofv3 --kernel-trace -d gpurun_out/r3aw_tl -o run --output-format csv -- python3 tools/kernel_ab.py --warmup 140 --steps 200
f=$(find gpurun_out/r3aw_tl -name '*kernel_trace.csv' | head -1)
python3 tools/step_timeline.py "$f" k_gather_ln_gmf 0.5 > gpurun_out/r3aw_timeline.txt
rm -f "$f"
cat gpurun_out/r3aw_timeline.txt
