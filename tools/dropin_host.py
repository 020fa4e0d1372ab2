#!/usr/bin/env python3
"""Host cost of the reference call pattern on the fused path (C2 shapes).

Times the host side of each phase of ``model(kjt) -> BCELoss -> zero_grad -> backward ->
Adam.step`` (no syncs: what the Python thread spends enqueueing), the GPU time per step, and a
cProfile of the loop (top functions by own time).  GPU box only.

    python tools/dropin_host.py [--steps 200] [--profile]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _ncf_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=160)
    ap.add_argument("--profile", action="store_true")
    a = ap.parse_args()
    ncf = _ncf_pkg.load()
    dev = torch.device("cuda:0")
    U, I, B, M = 1_000_000, 100_000, 4096, 5
    torch.manual_seed(0)
    m = ncf.AdvancedNCF(U, I, 10, 50, 64, 64, 32, [256, 128, 64], 4, 0.2, 4).to(dev).train()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-5)
    crit = torch.nn.BCELoss()
    g = torch.Generator(device=dev).manual_seed(1)
    feats = []
    for _ in range(8):
        u = torch.randint(0, U, (B,), generator=g, device=dev).repeat_interleave(M)
        i = torch.randint(0, I, (B * M,), generator=g, device=dev)
        t = torch.zeros(B, M, device=dev)
        t[:, 0] = 1
        kj = ncf.KeyedJaggedTensor.from_lengths_sync(
            keys=["user_id", "product_id"], values=torch.cat([u, i]),
            lengths=torch.ones(2 * B * M, dtype=torch.long, device=dev))
        feats.append((kj, t.reshape(-1, 1)))
    ph = {"forward": 0.0, "loss": 0.0, "zero_grad": 0.0, "backward": 0.0, "step": 0.0}

    def run(first, n, timed=False):
        for s in range(first, first + n):
            f, t = feats[s % len(feats)]
            t0 = time.perf_counter()
            out = m(f)
            t1 = time.perf_counter()
            loss = crit(out, t)
            t2 = time.perf_counter()
            opt.zero_grad()
            t3 = time.perf_counter()
            loss.backward()
            t4 = time.perf_counter()
            opt.step()
            t5 = time.perf_counter()
            if timed:
                for k, d in zip(ph, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4)):
                    ph[k] += d
    run(0, a.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(a.warmup, a.steps, timed=True)
    host = time.perf_counter() - t0
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    print(f"wall {wall / a.steps * 1e3:.4f} ms/step; host enqueue {host / a.steps * 1e3:.4f} ms/step")
    for k, v in ph.items():
        print(f"  {k:10s} {v / a.steps * 1e6:8.1f} us/step (host)")
    if a.profile:
        pr = cProfile.Profile()
        pr.enable()
        run(0, a.steps)
        pr.disable()
        torch.cuda.synchronize()
        pstats.Stats(pr).sort_stats("tottime").print_stats(35)


if __name__ == "__main__":
    main()
