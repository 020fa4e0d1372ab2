"""HBM bytes per launch per kernel from two rocprofv3 counter-collection passes.

    python tools/pmc_traffic.py <FETCH_SIZE dir> <WRITE_SIZE dir> <out.json>

MI355X_MICROARCH.md (HBM section): FETCH_SIZE / WRITE_SIZE come from the L2's memory-side
request counters and cannot share a pass; on gfx950 FETCH_SIZE reports exactly half the bytes of
a wide coalesced read, so it is doubled; both are in KiB (x1024).  The per-kernel value is the
mean over that kernel's launches in the run."""
import csv
import glob
import json
import os
import re
import sys


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    acc = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            m = re.search(r"\b(k_[A-Za-z0-9_]+)", r["Kernel_Name"])
            name = m.group(1) if m else r["Kernel_Name"][:40]
            key = (name, int(r["Grid_Size"]))
            v = float(r["Counter_Value"])
            s, n = acc.get(key, (0.0, 0))
            acc[key] = (s + v, n + 1)
    return {k: (s / n, n) for k, (s, n) in acc.items()}


def main():
    fd, wd, out = sys.argv[1:4]
    fetch = load(fd, "FETCH_SIZE")
    write = load(wd, "WRITE_SIZE")
    kernels = {}
    for key in sorted(set(fetch) | set(write)):
        name, grid = key
        f = fetch.get(key, (0.0, 0))[0] * 1024.0 * 2.0      # KiB -> B, gfx950 x2 correction
        w = write.get(key, (0.0, 0))[0] * 1024.0
        n = max(fetch.get(key, (0, 0))[1], write.get(key, (0, 0))[1])
        e = {"grid": grid, "launches": n, "fetch_bytes_per_launch": round(f),
             "write_bytes_per_launch": round(w), "hbm_bytes_per_launch": round(f + w)}
        kernels.setdefault(name, {"by_grid": []})["by_grid"].append(e)
    for name, k in kernels.items():   # headline entry: the grid carrying the most bytes overall
        best = max(k["by_grid"], key=lambda e: e["launches"] * (e["hbm_bytes_per_launch"] + 1))
        k.update({x: best[x] for x in ("grid", "fetch_bytes_per_launch", "write_bytes_per_launch",
                                       "hbm_bytes_per_launch")})
    with open(out, "w") as fh:
        json.dump({"method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes "
                             "over `bench.py --steps 5 --warmup 3`; FETCH_SIZE x2 (gfx950), KiB x1024; "
                             "mean per launch", "kernels": kernels}, fh, indent=1, sort_keys=True)
    for k, v in sorted(kernels.items()):
        print(f"{k:28s} grid {v['grid']:>9d}  fetch {v['fetch_bytes_per_launch'] / 1e6:9.3f} MB  "
              f"write {v['write_bytes_per_launch'] / 1e6:9.3f} MB")


if __name__ == "__main__":
    main()
