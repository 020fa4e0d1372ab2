#!/bin/bash
# Round-3: release scope of the step's stream-to-stream events (0 system / 1 device / 2 none):
# the GPU suite under 1 and 2, then interleaved fused-step and drop-in timings, then one step's
# per-queue timeline under the fastest.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; }; }
for sc in 1 2; do
NCF_EVENT_SCOPE=$sc step r3av_tests_$sc 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
echo "scope $sc: $(tail -1 gpurun_out/r3av_tests_$sc.log)"
done
for rep in 1 2; do
for sc in 0 1 2; do
NCF_EVENT_SCOPE=$sc step r3av_ab_${sc}_$rep 200 python3 -u tools/kernel_ab.py --tag scope$sc
NCF_EVENT_SCOPE=$sc step r3av_di_${sc}_$rep 200 python3 -u tools/dropin_host.py --warmup 150 --steps 300
echo "scope $sc: fused $(grep '^{' gpurun_out/r3av_ab_${sc}_$rep.log | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])') dropin $(grep -v amdgpu gpurun_out/r3av_di_${sc}_$rep.log | head -2 | tr '\n' ' ')"
done
done
for sc in 1 2; do
NCF_EVENT_SCOPE=$sc step r3av_tl_$sc 300 rocprofv3 --kernel-trace -d gpurun_out/r3av_tl_$sc -o run --output-format csv -- python3 tools/kernel_ab.py --warmup 140 --steps 200
f=$(find gpurun_out/r3av_tl_$sc -name '*kernel_trace.csv' | head -1)
python3 tools/step_timeline.py "$f" k_gather_ln_gmf 0.5 > gpurun_out/r3av_timeline_$sc.txt
rm -f "$f"
done
cat gpurun_out/r3av_timeline_1.txt
