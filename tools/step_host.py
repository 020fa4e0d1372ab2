"""Host-side cost of FusedTrainStep (pipelined, the bench's form) at a batch size: cProfile over
`--steps` steps after the deferred schedule's steady state (GPU only).

    python tools/step_host.py [--groups 256] [--steps 200]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _ncf_pkg  # noqa: E402
import bench  # noqa: E402

ncf = _ncf_pkg.load()
from ncf_amd.trainer import FusedTrainStep  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=256)
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    U, I, B, M = 1_000_000, 100_000, a.groups, 5
    torch.manual_seed(0)
    model = ncf.AdvancedNCF(U, I, 10, 50).to(dev).train()
    step = FusedTrainStep(model, lr=1e-3, weight_decay=1e-5)
    batches = bench.make_batches(U, I, B, M, 8, dev, seed=5)

    def run(first, count):
        for s in range(first, first + count):
            step(*batches[s % 8], next=batches[(s + 1) % 8][:2])
    run(0, 300)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(300, a.steps)
    th = time.perf_counter()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    print(f"host {1e3 * (th - t0) / a.steps:.4f} ms/step, wall {1e3 * (t1 - t0) / a.steps:.4f} "
          f"ms/step", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    run(300 + a.steps, a.steps)
    pr.disable()
    torch.cuda.synchronize()
    buf = io.StringIO()
    pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(35)
    pstats.Stats(pr, stream=buf).sort_stats("cumulative").print_stats(30)
    print(buf.getvalue())


if __name__ == "__main__":
    main()
