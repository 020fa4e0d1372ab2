"""Is the training step host-bound?  Times the host-side enqueue of K steps (no sync inside the
loop) against the synchronised wall time, at the C2 workload (GPU only).

    python tools/host_overhead.py [--steps 30]"""
import argparse
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda")
    U, I, B, M = 1_000_000, 100_000, 4096, 5
    torch.manual_seed(0)
    model = ncf.AdvancedNCF(U, I, 10, 50).to(dev).train()
    step = FusedTrainStep(model, lr=1e-3, weight_decay=1e-5)
    batches = bench.make_batches(U, I, B, M, 8, dev, seed=5)
    for s in range(5):
        step(*batches[s % 8])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(a.steps):
        step(*batches[s % 8])
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print(f"host enqueue {t_host / a.steps * 1e3:.3f} ms/step, wall {t_all / a.steps * 1e3:.3f} ms/step",
          flush=True)


if __name__ == "__main__":
    main()
