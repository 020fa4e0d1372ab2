#!/usr/bin/env python3
"""A/B the C2 training step between library builds (GPU box only).

    NCF_HIP_LIB=path/to/libncf_hip.so python tools/kernel_ab.py [--tag name]

Runs the headline step (FusedTrainStep, pipelined dedup) for a steady-state warm-up, times 200
steps, then 40 steps with per-launch HIP events; prints one JSON line: ms/step and the mean
microseconds per step of every C-ABI entry point.
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
from bench import make_batches  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default=os.environ.get("NCF_HIP_LIB", "default"))
    ap.add_argument("--warmup", type=int, default=140)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--bf16", action="store_true", help="bf16-table configuration")
    a = ap.parse_args()
    ncf = _ncf_pkg.load()
    from ncf_amd import _lib as L
    from ncf_amd.trainer import FusedTrainStep
    dev = torch.device("cuda:0")
    torch.manual_seed(1234)
    U, I, B, M = 1_000_000, 100_000, 4096, 5
    m = ncf.AdvancedNCF(U, I, 10, 50, 64, 64, 32, [256, 128, 64], 4, 0.2, 4).to(dev).train()
    step = FusedTrainStep(m, lr=1e-3, weight_decay=1e-5,
                          sweep_every=int(os.environ.get("AB_SWEEP_EVERY", "64")),
                          table_dtype=torch.bfloat16 if a.bf16 else torch.float32)
    batches = make_batches(U, I, B, M, 8, dev, seed=100)

    def run(first, n, pipe=True):
        for s in range(first, first + n):
            u, i, t = batches[s % 8]
            if pipe:
                step(u, i, t, next=batches[(s + 1) % 8][:2])
            else:
                step(u, i, t)
    run(0, a.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(a.warmup, a.steps)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.steps * 1e3
    L.PROFILE = []
    run(a.warmup + a.steps, 40, pipe=False)
    torch.cuda.synchronize()
    prof, L.PROFILE = L.PROFILE, None
    per = {}
    for name, _, e0, e1 in prof:
        per[name] = per.get(name, 0.0) + e0.elapsed_time(e1) * 1e3 / 40
    print(json.dumps({"tag": a.tag, "ms_per_step": round(ms, 4),
                      "us": {k: round(v, 1) for k, v in sorted(per.items(), key=lambda x: -x[1])},
                      "loss": round(float(step.last_loss.item()), 6)}), flush=True)


if __name__ == "__main__":
    main()
