#!/bin/bash
# Round-3: the next batch's id sort queued behind the overlapped sweep on its stream
# (NCF_DEDUP_FORK=sweep: no fork record on the step's queue) vs forked at the attention backward.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; }; }
step r3ax_tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/r3ax_tests.log
for rep in 1 2 3; do
for f in attn_bwd sweep; do
NCF_DEDUP_FORK=$f step r3ax_ab_${f}_$rep 200 python3 -u tools/kernel_ab.py --tag $f
echo "$f: fused $(grep '^{' gpurun_out/r3ax_ab_${f}_$rep.log | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
done
done
step r3ax_tl 300 rocprofv3 --kernel-trace -d gpurun_out/r3ax_tl -o run --output-format csv -- python3 tools/kernel_ab.py --warmup 140 --steps 200
f=$(find gpurun_out/r3ax_tl -name '*kernel_trace.csv' | head -1)
python3 tools/step_timeline.py "$f" k_gather_ln_gmf 0.5 > gpurun_out/r3ax_timeline.txt
rm -f "$f"
cat gpurun_out/r3ax_timeline.txt
