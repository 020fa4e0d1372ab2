"""Per-launch times of the fused tower / attention kernels in the C2 step (GPU only): the fp32
step with the tower on fp32 MFMA and on split-operand bf16 MFMA (engine.TOWER_SPLIT), and the
bf16-table step (single-term bf16 MFMA), with the rolling sweep on the step's own stream
(kernels not sharing the CUs with it); also the step time of each.
    python tools/tower_ab.py [--steps 40]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _ncf_pkg  # noqa: E402
import bench  # noqa: E402

ncf = _ncf_pkg.load()
from ncf_amd import _lib  # noqa: E402
from ncf_amd.trainer import FusedTrainStep  # noqa: E402

NAMES = ("ncf_attn_mlp_fwd", "ncf_attn_mlp_bwd", "ncf_mlp_bwd", "ncf_mlp_bwd_split", "ncf_mlp_bwd_bf16", "ncf_mlp_fwd", "ncf_mlp_fwd_split",
         "ncf_mlp_fwd_bf16", "ncf_attn_block_fwd",
         "ncf_attn_block_bwd", "ncf_reduce_batch", "ncf_embedding_bwd_reduce",
         "ncf_gather_ln_gmf_scaled_fwd", "ncf_adam_pairs_apply_clock", "ncf_adam_pairs_catchup_clock", "ncf_adam_pairs_catchup_lock_clock",
         "ncf_adam_flat_clock_close")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    U, I, D, B, M = 1_000_000, 100_000, 64, 4096, 5
    batches = bench.make_batches(U, I, B, M, 16, dev, seed=3)
    import ncf_amd.engine as E
    for dt, split in ((torch.float32, False), (torch.float32, True), (torch.bfloat16, False)):
        E.TOWER_SPLIT = split
        torch.manual_seed(5)
        m = ncf.AdvancedNCF(U, I, 10, 50, D, D, 32, [256, 128, 64], 4, 0.2, M - 1).to(dev).train()
        step = FusedTrainStep(m, lr=1e-3, weight_decay=1e-5, table_dtype=dt)
        step.deferred.overlap = False

        def run(first, count):
            for s in range(first, first + count):
                u, i, t = batches[s % len(batches)]
                step(u, i, t, next=batches[(s + 1) % len(batches)][:2])
        run(0, 20)
        torch.cuda.synchronize()
        import time
        t0 = time.perf_counter()
        run(20, args.steps)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / args.steps * 1e3
        _lib.PROFILE = []
        run(20, args.steps)
        torch.cuda.synchronize()
        prof, _lib.PROFILE = _lib.PROFILE, None
        per = {}
        for name, _, e0, e1 in prof:
            per.setdefault(name, []).append(e0.elapsed_time(e1) * 1e3)
        print(f"== tables {dt}, split tower {split}: {ms:.4f} ms/step (sweep not overlapped)")
        for k in NAMES:
            if k in per:
                v = sorted(per[k])
                print(f"  {k:34s} median {v[len(v) // 2]:7.1f} us  min {v[0]:7.1f}  "
                      f"({len(v) / args.steps:.0f}/step)", flush=True)
        del step, m
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
