#!/bin/bash
# Round-3: the overlapped sweep's join as a stream-ordered device-word write / wait
# (NCF_JOIN_FLAG=1) against the event record / wait: GPU suite under the flag join, then
# interleaved fused-step A/B and one step's per-queue timeline with it.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; }; }
NCF_JOIN_FLAG=1 step r3ay_tests 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
tail -1 gpurun_out/r3ay_tests.log
for rep in 1 2 3; do
for f in 0 1; do
NCF_JOIN_FLAG=$f step r3ay_ab_${f}_$rep 200 python3 -u tools/kernel_ab.py --tag f$f
echo "flag=$f: fused $(grep '^{' gpurun_out/r3ay_ab_${f}_$rep.log | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
done
done
for f in 0 1; do
NCF_JOIN_FLAG=$f step r3ay_bench_$f 300 python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-score --no-c4
echo "flag=$f bench: $(grep '^{' gpurun_out/r3ay_bench_$f.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["dropin_train"]["ms_per_step"], d["c2_bf16_tables"]["ms_per_step"])')"
done
NCF_JOIN_FLAG=1 step r3ay_tl 300 rocprofv3 --kernel-trace -d gpurun_out/r3ay_tl -o run --output-format csv -- python3 tools/kernel_ab.py --warmup 140 --steps 200
f=$(find gpurun_out/r3ay_tl -name '*kernel_trace.csv' | head -1)
python3 tools/step_timeline.py "$f" k_gather_ln_gmf 0.5 > gpurun_out/r3ay_timeline.txt
rm -f "$f"
tail -22 gpurun_out/r3ay_timeline.txt
