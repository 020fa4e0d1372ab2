"""One step's kernels from a rocprofv3 kernel-trace CSV with their start offsets, durations,
queues and the idle gap before each kernel on its queue (where the critical path waits).
    python tools/step_timeline.py TRACE.csv [anchor kernel] [fraction of the run]"""
import csv
import sys

path = sys.argv[1]
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_gather_ln_gmf"
frac = float(sys.argv[3]) if len(sys.argv) > 3 else 0.5


def short(name):
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return name.split("(")[0].split("<")[0]


rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]).startswith(anchor)]
j = int(len(idx) * frac)
a, b = idx[j], idx[j + 1]
t0 = int(rows[a]["Start_Timestamp"])
last_end = {}
qs = {}
print(f"{'kernel':34s} {'queue':>5s} {'start':>8s} {'dur':>7s} {'end':>8s} {'gap':>6s}")
for r in rows[a:b + 1]:
    q = r.get("Queue_Id", "?")
    qs.setdefault(q, len(qs))
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    gap = (s - last_end[q]) / 1e3 if q in last_end else 0.0
    last_end[q] = e
    print(f"{short(r['Kernel_Name'])[:34]:34s} {qs[q]:5d} {s / 1e3:8.1f} {(e - s) / 1e3:7.1f} "
          f"{e / 1e3:8.1f} {gap:6.1f}")
print(f"step span (anchor to anchor): {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us")
