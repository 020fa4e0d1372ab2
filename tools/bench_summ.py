"""One line per bench log: ms/step and selected per-entry-point times (ms/step).
    python tools/bench_summ.py LOG [TAG=value] [entry_point ...]   (no entry points: all)"""
import json
import sys

log = sys.argv[1]
d = [json.loads(l) for l in open(log) if l.startswith("{")][-1]
k = d.get("kernel_ms_per_step", {})
out = [log.split("/")[-1], f"{d['ms_per_step']:.4f}"]
names = [a for a in sys.argv[2:] if "=" not in a]
out += [a for a in sys.argv[2:] if "=" in a]
for name in names or sorted(k, key=lambda x: -k[x]):
    v = k.get(name)
    out.append(f"{name.replace('ncf_', '')}={v * 1e3:.1f}us" if v else f"{name}=-")
r = d.get("roofline", {})
if r:
    out.append(f"frac={r.get('frac')} iso={r.get('isolated', {}).get('ms_per_launch')}")
if isinstance(d.get("dropin_train"), dict):
    out.append(f"dropin={d['dropin_train']['ms_per_step']}")
print(" ".join(out))
