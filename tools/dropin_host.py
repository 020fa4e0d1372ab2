"""Host-side cost of the reference call pattern (model(kjt) -> BCELoss -> zero_grad -> backward ->
Adam.step) at C2: cProfile over `--steps` steps after a warm-up, the top functions by own time.
The drop-in path is host-bound when its host time per step exceeds the GPU's.

    python tools/dropin_host.py [--warmup 150] [--steps 100]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--warmup", type=int, default=150)
    ap.add_argument("--steps", type=int, default=100)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    ncf = _ncf_pkg.load()
    U, I, D, T, H, hid, B, M = 1_000_000, 100_000, 64, 32, 4, [256, 128, 64], 4096, 5
    torch.manual_seed(1234)
    m = ncf.AdvancedNCF(U, I, 10, 50, D, D, T, hid, H, 0.2, M - 1).to(dev).train()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-5)
    crit = torch.nn.BCELoss()
    feats = []
    for u, i, t in bench.make_batches(U, I, B, M, 8, dev, seed=100):
        kj = ncf.KeyedJaggedTensor.from_lengths_sync(
            keys=["user_id", "product_id"], values=torch.cat([u, i]),
            lengths=torch.ones(2 * u.numel(), dtype=torch.long, device=dev))
        feats.append((kj, t))

    def one(s):
        f, t = feats[s % len(feats)]
        out = m(f)
        loss = crit(out, t)
        opt.zero_grad()
        loss.backward()
        opt.step()

    for s in range(args.warmup):
        one(s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        one(s)
    th = time.perf_counter()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    print(f"host {1e3 * (th - t0) / args.steps:.4f} ms/step, wall {1e3 * (t1 - t0) / args.steps:.4f} ms/step"
          f" (launch tapes: {m.engine.tapes.replays} phases replayed, {m.engine.tapes.recorded} recorded)")
    # the backward on the calling thread, so the profile sees it (autograd otherwise runs it on
    # its device thread); timed that way too
    torch.autograd.set_multithreading_enabled(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        one(s)
    th = time.perf_counter()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    print(f"autograd on the calling thread: host {1e3 * (th - t0) / args.steps:.4f} ms/step, "
          f"wall {1e3 * (t1 - t0) / args.steps:.4f} ms/step")
    pr = cProfile.Profile()
    pr.enable()
    for s in range(args.steps):
        one(s)
    pr.disable()
    torch.cuda.synchronize()
    buf = io.StringIO()
    pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(30)
    pstats.Stats(pr, stream=buf).sort_stats("cumulative").print_stats(30)
    print(buf.getvalue())


if __name__ == "__main__":
    main()
