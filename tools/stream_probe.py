"""Does the C2 step's time depend on which hardware queue its side stream lands on?  Builds a
fresh FusedTrainStep after taking k streams from torch's per-device stream pool (k = 0..7: the
step's own side stream is then the pool's (k+1)-th), times 100 steps each (GPU only).
    python tools/stream_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _ncf_pkg  # noqa: E402
import bench  # noqa: E402

ncf = _ncf_pkg.load()
from ncf_amd.trainer import FusedTrainStep  # noqa: E402


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--priority", type=int, default=None,
                    help="deferred.SIDE_PRIORITY for the side streams (default: the module's)")
    ap.add_argument("--builds", type=int, default=16)
    a = ap.parse_args()
    from ncf_amd import deferred as Dm
    if a.priority is not None:
        Dm.SIDE_PRIORITY = a.priority
    print(f"side stream priority {Dm.SIDE_PRIORITY}", flush=True)
    dev = torch.device("cuda", 0)
    U, I, D, B, M = 1_000_000, 100_000, 64, 4096, 5
    batches = bench.make_batches(U, I, B, M, 64, dev, seed=3)
    for k in [j % 8 for j in range(a.builds)]:
        held = [torch.cuda.Stream(dev) for _ in range(k)]
        torch.manual_seed(5)
        model = ncf.AdvancedNCF(U, I, 10, 50, D, D, 32, [256, 128, 64], 4, 0.2, M - 1).to(dev).train()
        step = FusedTrainStep(model, lr=1e-3, weight_decay=1e-5)

        def run(first, count):
            for s in range(first, first + count):
                u, i, t = batches[s % len(batches)]
                step(u, i, t, next=batches[(s + 1) % len(batches)][:2])
        run(0, 140)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(140, 100)
        torch.cuda.synchronize()
        side = step.deferred._side
        ms = (time.perf_counter() - t0) / 100 * 1e3
        from ncf_amd import _lib
        _lib.PROFILE = []
        run(240, 20)
        torch.cuda.synchronize()
        prof, _lib.PROFILE = _lib.PROFILE, None
        per = {}
        for nm, _, e0, e1 in prof:
            per[nm] = per.get(nm, 0.0) + e0.elapsed_time(e1) * 1e3 / 20
        top = " ".join(f"{k_[4:18]}={v:.0f}" for k_, v in sorted(per.items(), key=lambda x: -x[1])[:7])
        print(f"k={k} side stream {side.cuda_stream:#x}: {ms:.4f} ms/step | {top}", flush=True)
        del step, model, held
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
