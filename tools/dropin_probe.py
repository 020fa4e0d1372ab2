"""Reproduce the drop-in leg of bench.py as the driver runs it (--steps 20 --warmup 5) and show
where its time goes: per-step wall times (each step synchronised) over the first steps, then the
async windowed rate, with the fused headline model alive beside it as in bench.py.

    python tools/dropin_probe.py [--warmup 5] [--steps 20] [--fused-first 25] [--trace 40]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _ncf_pkg  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--fused-first", type=int, default=25)
    ap.add_argument("--trace", type=int, default=40)
    ap.add_argument("--windows", type=int, default=6)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    ncf = _ncf_pkg.load()
    from ncf_amd.trainer import FusedTrainStep
    U, I, D, T, H, hid, B, M = 1_000_000, 100_000, 64, 32, 4, [256, 128, 64], 4096, 5
    torch.manual_seed(1234)
    model = ncf.AdvancedNCF(U, I, 10, 50, D, D, T, hid, H, 0.2, M - 1).to(dev).train()
    step = FusedTrainStep(model, lr=1e-3, weight_decay=1e-5)
    batches = bench.make_batches(U, I, B, M, 8, dev, seed=100)
    for s in range(args.fused_first):
        u, i, t = batches[s % 8]
        step(u, i, t, next=batches[(s + 1) % 8][:2])
    torch.cuda.synchronize()

    torch.manual_seed(1234)
    m = ncf.AdvancedNCF(U, I, 10, 50, D, D, T, hid, H, 0.2, M - 1).to(dev).train()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-5)
    crit = torch.nn.BCELoss()
    feats = []
    for u, i, t in batches:
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
        return loss

    rec = {"per_step_sync_ms": [], "per_step_host_ms": []}
    for s in range(args.trace):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        one(s)
        th = time.perf_counter()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        rec["per_step_sync_ms"].append(round((t1 - t0) * 1e3, 3))
        rec["per_step_host_ms"].append(round((th - t0) * 1e3, 3))
    s0 = args.trace
    win = []
    for k in range(args.windows):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in range(s0, s0 + args.steps):
            one(s)
        torch.cuda.synchronize()
        win.append(round((time.perf_counter() - t0) / args.steps * 1e3, 4))
        s0 += args.steps
    rec["async_window_ms"] = win
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
