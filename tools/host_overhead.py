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
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--pipe", action="store_true", help="pipelined dedup (next=, the bench's form)")
    ap.add_argument("--groups", type=int, default=4096, help="B (256: the reference's batch)")
    ap.add_argument("--graph", action="store_true", help="FusedTrainStep(graph=True): hipGraph replay")
    a = ap.parse_args()
    dev = torch.device("cuda")
    U, I, B, M = 1_000_000, 100_000, a.groups, 5
    torch.manual_seed(0)
    model = ncf.AdvancedNCF(U, I, 10, 50).to(dev).train()
    step = FusedTrainStep(model, lr=1e-3, weight_decay=1e-5, graph=a.graph)
    batches = bench.make_batches(U, I, B, M, 8, dev, seed=5)
    def one(s):
        if a.pipe and not a.graph:
            step(*batches[s % 8], next=batches[(s + 1) % 8][:2])
        else:
            step(*batches[s % 8])
    for s in range(max(a.warmup, 300)):      # (the deferred schedule's steady state)
        one(s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    w0 = max(a.warmup, 300)
    for s in range(w0, w0 + a.steps):
        one(s)
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print(f"host enqueue {t_host / a.steps * 1e3:.3f} ms/step, wall {t_all / a.steps * 1e3:.3f} ms/step",
          flush=True)


if __name__ == "__main__":
    main()
