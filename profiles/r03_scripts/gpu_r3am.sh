#!/bin/bash
# Round-3: C5 item split sized from the expected candidates per user: tests, time, writes.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -30 "gpurun_out/$name.log"; exit $rc; }; }
step r3am_tests 400 python3 -u -m pytest tests/test_gpu_parity.py -k "scor or topk or score" -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/r3am_tests.log
step r3am_t 200 python3 -u tools/score_bench.py --reps 3
grep -v amdgpu gpurun_out/r3am_t.log | head -4
for C in FETCH_SIZE WRITE_SIZE; do
  step r3am_pmc_$C 200 rocprofv3 --pmc $C -d gpurun_out/r3am_pmc_$C -o run --output-format csv -- python3 tools/score_bench.py --reps 1
done
python3 tools/pmc_traffic.py gpurun_out/r3am_pmc_FETCH_SIZE gpurun_out/r3am_pmc_WRITE_SIZE gpurun_out/r3am_c5_pmc_traffic.json | grep -i "collect3\|select"
f=$(find gpurun_out/r3am_pmc_WRITE_SIZE -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
vals = [round(float(r["Counter_Value"]) * 1024 / 1e6, 1) for r in csv.DictReader(open(sys.argv[1])) if "k_collect3" in r["Kernel_Name"]]
print("  k_collect3 WRITE_SIZE per launch (MB):", vals)
PY
