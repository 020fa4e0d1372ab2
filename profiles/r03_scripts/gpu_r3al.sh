#!/bin/bash
# Round-3: C5 scan rounds (item splits) vs k_collect3 write traffic and time.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -30 "gpurun_out/$name.log"; exit $rc; }; }
for R in 4 8 16; do
  echo "rounds $R"
  NCF_SCORE3_ROUNDS=$R step r3al_w$R 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r3al_pmcw$R -o run --output-format csv -- python3 tools/score_bench.py --reps 1
  f=$(find gpurun_out/r3al_pmcw$R -name '*counter_collection.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, sys
vals = []
for r in csv.DictReader(open(sys.argv[1])):
    if "k_collect3" in r["Kernel_Name"]:
        vals.append(float(r["Counter_Value"]) * 1024 / 1e6)
print("  k_collect3 WRITE_SIZE per launch (MB):", [round(v, 1) for v in vals])
PY
done
