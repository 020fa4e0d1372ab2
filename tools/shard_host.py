"""Host cost of the row-sharded step (world size 1 over RCCL, GPU only): wall ms/step, and a
cProfile of K steps (top functions by own time) to show where the host spends its time.

    python tools/shard_host.py [--steps 30]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _ncf_pkg  # noqa: E402
import bench  # noqa: E402

ncf = _ncf_pkg.load()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    dist.init_process_group("nccl", rank=0, world_size=1)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from ncf_amd.distributed import make_sharded_step
    U, I, B, M = 1_000_000, 100_000, 4096, 5

    def factory(ru, ri):
        torch.manual_seed(0)
        return ncf.AdvancedNCF(ru, ri, 10, 50).to(dev).train()
    model, step = make_sharded_step(factory, U, I, lr=1e-3, weight_decay=1e-5)
    batches = bench.make_batches(U, I, B, M, 8, dev, seed=5)

    def run(first, k):
        for s in range(first, first + k):
            u, i, t = batches[s % 8]
            step(u, i, t, next=batches[(s + 1) % 8][:2])
    run(0, 5)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(5, a.steps)
    th = time.perf_counter()
    torch.cuda.synchronize()
    T = step.tapes
    print(f"wall {(time.perf_counter() - t0) / a.steps * 1e3:.3f} ms/step, host "
          f"{(th - t0) / a.steps * 1e3:.3f} ms/step; launch tapes: "
          + (f"{T.replays} segments replayed, {T.recorded} recorded, keys {sorted(T.entries)}"
             if T is not None else "off"), flush=True)
    # host time per protocol phase (wrappers on the ops / exchange methods)
    acc = {}

    def wrap(obj, name, label=None):
        fn = getattr(obj, name)

        def timed(*x, **k):
            t = time.perf_counter()
            r = fn(*x, **k)
            acc[label or name] = acc.get(label or name, 0.0) + time.perf_counter() - t
            return r
        setattr(obj, name, timed)
    for nm in ("plan", "owner_prepare", "owner_gather", "compute", "owner_apply", "dense_step"):
        wrap(step.ops, nm)
    for nm in ("exchange_counts", "exchange", "all_reduce_"):
        wrap(step.x, nm)
    wrap(step.ops.eng, "forward", "compute.forward")
    wrap(step.ops.eng, "backward", "compute.backward")
    t0 = time.perf_counter()
    run(5 + a.steps, a.steps)
    host = time.perf_counter() - t0
    torch.cuda.synchronize()
    print(f"instrumented: host {host / a.steps * 1e3:.3f} ms/step; per phase (us/step):", flush=True)
    for k, v in sorted(acc.items(), key=lambda x: -x[1]):
        print(f"  {k:24s} {v / a.steps * 1e6:8.1f}")
    pr = cProfile.Profile()
    pr.enable()
    run(5 + 2 * a.steps, a.steps)
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
