#!/usr/bin/env python3
"""Per-kernel mean of every SQ counter collected by tools/pmc_sq.sh (rocprofv3 csv)."""
import csv
import glob
import sys
from collections import defaultdict

tag = sys.argv[1] if len(sys.argv) > 1 else ""
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"gpurun_out/sq{tag}_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        k = k.split("(")[0].split("<")[0][:40]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(acc.items()):
    keys = sys.argv[2].split(",") if len(sys.argv) > 2 else (
        "mlp", "attn", "gather", "piece", "reduce", "pairs", "dedup")
    if not any(x in k for x in keys):
        continue
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.0f}")
