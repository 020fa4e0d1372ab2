"""Summarise a rocprofv3 kernel-trace CSV: per-kernel totals and one step's timeline."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_gather_ln_gmf"
def short(name):
    """'void (anonymous namespace)::k_mlp_bwd<false>(float const*, ...)' -> 'k_mlp_bwd'"""
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return name.split("(")[0].split("<")[0]


rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
for r in rows:
    r["Kernel_Name"] = short(r["Kernel_Name"])
idx = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(anchor)]
a, b = idx[len(idx) // 2], idx[len(idx) // 2 + 1]
tot = 0.0
agg = {}
for r in rows[a:b]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    k = r["Kernel_Name"][:40]
    agg[k] = agg.get(k, 0.0) + d
    if "-v" in sys.argv:
        print(f"{k:40s} grid={r['Grid_Size_X']:>8s}x{r['Grid_Size_Y']:>3s}x{r['Grid_Size_Z']:>4s} {d:8.2f} us")
span = (int(rows[b - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
print(f"one step: {b - a} kernels, sum of kernel time {tot:.1f} us, wall span {span:.1f} us")
for k, v in sorted(agg.items(), key=lambda x: -x[1])[:25]:
    print(f"  {k:40s} {v:8.1f} us")
