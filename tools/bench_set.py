"""bench.py with ncf_amd module constants overridden first (A/B of a constant on any bench leg,
torchrun included):
    python tools/bench_set.py --set distributed.SWEEP_EVERY=128 -- --sharded --steps 200
    python -m torch.distributed.run --nproc-per-node 1 ... tools/bench_set.py --set ... -- --sharded"""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    argv = sys.argv[1:]
    rest = argv[argv.index("--") + 1:] if "--" in argv else []
    own = argv[:argv.index("--")] if "--" in argv else argv
    sets = [a for a in own if a != "--set"]
    import _ncf_pkg
    _ncf_pkg.load()
    for spec in sets:
        path, _, val = spec.partition("=")
        mod, _, const = path.rpartition(".")
        m = importlib.import_module("ncf_amd." + mod)
        old = getattr(m, const)
        setattr(m, const, type(old)(int(val)) if isinstance(old, (bool, int)) else type(old)(val))
        print(f"set {path} = {getattr(m, const)!r}", file=sys.stderr, flush=True)
    import bench
    sys.argv = [os.path.join(ROOT, "bench.py")] + rest
    bench.main()


if __name__ == "__main__":
    main()
