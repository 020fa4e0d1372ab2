"""C2 step time (the bench's training step: FusedTrainStep with next=, overlapped sweep, 256
resident Zipf batches) under module-constant variants, interleaved in one process so the box's
drift hits every variant alike (GPU only).
    python tools/step_ab.py [--steps 200] [--reps 3] [--groups 4096] VARIANT [VARIANT ...]
VARIANT: name=module.CONST:value[,module.CONST:value][,sweep:N][,env:NAME:value][,c:SETTER:v]
(c: a C-ABI setter taking one int64, e.g. c:ncf_reduce_set_vec:0, restored after the variant)  e.g.
    base=engine.FUSE_ATTN_TOWER:1  nofuse=engine.FUSE_ATTN_TOWER:0  noearly=deferred.EARLY_CATCHUP:0
Per variant: ms/step of each repetition and the per-entry-point ms/step of one profiled run."""
import argparse
import importlib
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _ncf_pkg  # noqa: E402
import bench  # noqa: E402

ncf = _ncf_pkg.load()
from ncf_amd import _lib  # noqa: E402
from ncf_amd.trainer import FusedTrainStep  # noqa: E402


def parse(spec):
    """-> (name, [(module, const, value)], FusedTrainStep kwargs); ``sweep:N`` sets sweep_every."""
    name, _, body = spec.partition("=")
    sets, kw = [], {}
    for item in filter(None, body.split(",")):
        path, _, val = item.partition(":")
        if path == "sweep":
            kw["sweep_every"] = int(val)
            continue
        if path == "prio":    # prio:P: the steps run on a stream of priority P
            kw["_prio"] = int(val)
            continue
        if path == "c":       # c:SETTER:value (a C-ABI setter, int64 in, previous value out)
            fn, _, v = val.partition(":")
            kw.setdefault("_c", []).append((fn, int(v)))
            continue
        if path == "env":     # env:NAME:value ('+' for ',' inside the value)
            k, _, v = val.partition(":")
            kw.setdefault("_env", {})[k] = v.replace("+", ",")
            continue
        mod, _, const = path.rpartition(".")
        m = importlib.import_module("ncf_amd." + mod)
        old = getattr(m, const)
        if isinstance(old, (bool, int)):
            v = type(old)(int(val))
        elif old is None and (val == "None" or val.lstrip("-").isdigit()):
            v = None if val == "None" else bool(int(val))    # (a tri-state switch: None / 0 / 1)
        elif old is None or isinstance(old, str):    # ('+' for ',' inside a string value)
            v = val.replace("+", ",")
        else:
            v = type(old)(val)
        sets.append((m, const, v))
    return name, sets, kw


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--groups", type=int, default=4096, help="B (4096: C2; 256: the reference's)")
    ap.add_argument("variants", nargs="+")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    U, I, D, B, M = 1_000_000, 100_000, 64, args.groups, 5
    batches = bench.make_batches(U, I, B, M, 256, dev, seed=3)
    variants = [parse(v) for v in args.variants]
    defaults = {(m, c): getattr(m, c) for _, sets, _ in variants for m, c, _ in sets}
    res = {name: [] for name, _, _ in variants}
    prof = {}
    for rep in range(args.reps):
        for name, sets, kw in variants:
            for (m, c), v in defaults.items():
                setattr(m, c, v)
            for m, c, v in sets:
                setattr(m, c, v)
            csaved = [(fn, _lib.query(fn, v)) for fn, v in kw.get("_c", [])]
            env = kw.get("_env", {})
            saved = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            torch.manual_seed(5)
            model = ncf.AdvancedNCF(U, I, 10, 50, D, D, 32, [256, 128, 64], 4, 0.2, M - 1).to(dev).train()
            step = FusedTrainStep(model, lr=1e-3, weight_decay=1e-5,
                                  **{k: v for k, v in kw.items() if not k.startswith("_")})
            prio = kw.get("_prio")
            pstream = torch.cuda.Stream(dev, priority=prio) if prio is not None else None
            if pstream is not None:
                pstream.wait_stream(torch.cuda.current_stream(dev))
                torch.cuda.set_stream(pstream)
            for k, v in saved.items():     # (read by the constructors above only)
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v

            def run(first, count):
                for s in range(first, first + count):
                    u, i, t = batches[s % len(batches)]
                    step(u, i, t, next=batches[(s + 1) % len(batches)][:2])
            # (the deferred schedule's steady state: 2 x sweep_every steps, bench.py's prime)
            p0 = max(150, 2 * int(step.deferred.sweep_every if step.deferred else 0) + 20)
            run(0, p0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(p0, args.steps)
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / args.steps * 1e3)
            if rep == 0:
                _lib.PROFILE = []
                run(p0 + args.steps, 20)
                torch.cuda.synchronize()
                p, _lib.PROFILE = _lib.PROFILE, None
                per = {}
                for nm, _, e0, e1 in p:
                    per[nm] = per.get(nm, 0.0) + e0.elapsed_time(e1) * 1e3 / 20
                prof[name] = per
            print(f"rep {rep} {name:12s} {res[name][-1]:.4f} ms/step", flush=True)
            if pstream is not None:
                torch.cuda.synchronize()
                torch.cuda.set_stream(torch.cuda.default_stream(dev))
            del step, model
            torch.cuda.empty_cache()
            for fn, v in reversed(csaved):
                _lib.query(fn, v)
    for name, _, _ in variants:
        v = sorted(res[name])
        print(f"== {name:12s} ms/step {' '.join(f'{x:.4f}' for x in res[name])}  min {v[0]:.4f}")
        for k, us in sorted(prof[name].items(), key=lambda x: -x[1]):
            if us >= 1.0:
                print(f"     {k:40s} {us:7.1f} us/step")


if __name__ == "__main__":
    main()
