#!/usr/bin/env python3
"""Kernel statistics and a kernel trace from a rocprofv3 database (run_results.db, the output
when no --output-format is given): the same columns as rocprofv3's kernel_stats.csv and
kernel_trace.csv, for the kernels (and step timelines, tools/step_timeline.py) this repo profiles.

    python tools/rocpd_stats.py DB [--stats OUT.csv] [--trace OUT.csv] [--top N]
"""
import argparse
import csv
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--stats")
    ap.add_argument("--trace")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, queue_id, grid_x, workgroup_x, vgpr_count, "
                     "accum_vgpr_count, lds_size, scratch_size from kernels order by start").fetchall()
    agg = {}
    for name, s, e, *_ in rows:
        d = agg.setdefault(name, [0, 0, None, 0])
        dur = e - s
        d[0] += 1
        d[1] += dur
        d[2] = dur if d[2] is None else min(d[2], dur)
        d[3] = max(d[3], dur)
    total = sum(v[1] for v in agg.values()) or 1
    order = sorted(agg.items(), key=lambda kv: -kv[1][1])
    if a.stats:
        with open(a.stats, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs",
                        "MaxNs"])
            for name, (n, tot, mn, mx) in order:
                w.writerow([name, n, tot, round(tot / n, 1), round(100.0 * tot / total, 4), mn, mx])
    if a.trace:
        with open(a.trace, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Queue_Id", "Grid_Size",
                        "Workgroup_Size", "VGPR_Count", "Accum_VGPR_Count", "LDS_Block_Size",
                        "Scratch_Size"])
            for r in rows:
                w.writerow(list(r))
    for name, (n, tot, mn, mx) in order[:a.top]:
        short = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        print(f"{short[:60]:60s} {n:7d} {tot / n / 1e3:9.2f} us  {100.0 * tot / total:6.2f}%")


if __name__ == "__main__":
    main()
