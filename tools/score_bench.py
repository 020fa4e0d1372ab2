"""C5 scoring micro-benchmark (GPU only): 10K users x 1M items top-K through ncf_amd.scoring.

    python tools/score_bench.py [--users 10000] [--items 1000000] [--k 10 100] [--graph]
        [--set scoring.CONST=value ...]
Prints per-stage device times and pairs/s (eager), and with --graph the GraphedScorer time (the
bench's C5 line).  --set overrides ncf_amd module constants before anything runs (A/B)."""
import importlib
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _ncf_pkg  # noqa: E402

ncf = _ncf_pkg.load()
from ncf_amd import _lib  # noqa: E402
from ncf_amd.scoring import GraphedScorer, ItemIndex, score_topk  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=10000)
    ap.add_argument("--items", type=int, default=1000000)
    ap.add_argument("--num-users", type=int, default=1000000)
    ap.add_argument("--k", type=int, nargs="+", default=[10, 100])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--graph", action="store_true")
    ap.add_argument("--set", nargs="*", default=[])
    a = ap.parse_args()
    for spec in a.set:
        path, _, val = spec.partition("=")
        mod, _, const = path.rpartition(".")
        mm = importlib.import_module("ncf_amd." + mod)
        old = getattr(mm, const)
        setattr(mm, const, type(old)(int(val)) if isinstance(old, (bool, int)) else type(old)(val))
        print(f"set {path} = {getattr(mm, const)!r}", flush=True)
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = ncf.AdvancedNCF(a.num_users, a.items, 5, 24).to(dev)
    m.eval()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    idx = ItemIndex(m)
    torch.cuda.synchronize()
    print(f"item index ({a.items} items): {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
    for _ in range(2):   # a rebuild after a parameter change (warm caches and workspaces)
        _lib.PROFILE = []
        t0 = time.perf_counter()
        idx = ItemIndex(m)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        prof, _lib.PROFILE = _lib.PROFILE, None
        per = {}
        for name, _, e0, e1 in prof:
            per[name] = per.get(name, 0.0) + e0.elapsed_time(e1)
        print(f"item index rebuild: {dt * 1e3:.2f} ms  "
              + " ".join(f"{n}={v:.2f}ms" for n, v in per.items()), flush=True)
    users = torch.randperm(a.num_users, device=dev)[:a.users]
    for k in a.k:
        score_topk(m, users, k, idx)
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(a.reps):
            _lib.PROFILE = []
            t0 = time.perf_counter()
            s, it = score_topk(m, users, k, idx)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            prof, _lib.PROFILE = _lib.PROFILE, None
            best = min(best, dt)
        per = {}
        for name, _, e0, e1 in prof:
            per[name] = per.get(name, 0.0) + e0.elapsed_time(e1)
        pairs = a.users * a.items
        print(f"k={k}: {best * 1e3:.2f} ms  {pairs / best / 1e9:.1f} G pairs/s  "
              + " ".join(f"{n}={v:.2f}ms" for n, v in per.items()), flush=True)
        if a.graph:
            sc = GraphedScorer(m, n_users=a.users, k=k, index=idx)
            sc(users, copy=False)
            torch.cuda.synchronize()
            g = 1e9
            for _ in range(max(3, a.reps)):
                t0 = time.perf_counter()
                sc(users, copy=False)
                torch.cuda.synchronize()
                g = min(g, time.perf_counter() - t0)
            print(f"k={k}: graphed {g * 1e3:.3f} ms", flush=True)
            del sc


if __name__ == "__main__":
    main()
