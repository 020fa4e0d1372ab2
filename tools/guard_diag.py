"""Triage of test_guarded_fused_step_mixed_groups_ragged's failing case (GPU only): the same run
step by step, the device drained and the engine's id flag read after every step, the batch id
tensors compared with host copies (were they overwritten?), and the dedup outputs checked
(unique ids within range, counts plausible).

    python tools/guard_diag.py [--fuse-apply 0|1] [--early-reduce 0|1] [--pipelined 0|1]
                               [--guard 0|1] [--steps 6] [--sync-each 0|1]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _ncf_pkg  # noqa: E402
from tests.guard_alloc import guarded  # noqa: E402

ncf = _ncf_pkg.load()
DEV = torch.device("cuda:0")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fuse-apply", type=int, default=0)
    ap.add_argument("--early-reduce", type=int, default=0)
    ap.add_argument("--pipelined", type=int, default=0)
    ap.add_argument("--guard", type=int, default=1)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--sync-each", type=int, default=1)
    ap.add_argument("--log", default=None)
    a = ap.parse_args()
    import ncf_amd.trainer as Tr
    from ncf_amd import engine as E
    Tr.FUSE_APPLY = bool(a.fuse_apply)
    Tr.EARLY_REDUCE = bool(a.early_reduce)
    E.GROUP_ROWS = True
    U, I, B, M = 3000, 500, 61, 5
    torch.manual_seed(24)
    m = ncf.AdvancedNCF(U, I, 5, 24, 64, 64, 32, [256, 128, 64], 4, 0.2, M - 1).to(DEV)
    import contextlib
    ctx = guarded(log=a.log) if a.guard else contextlib.nullcontext()
    with ctx as arena:
        copy = arena.copy if a.guard else (lambda t: t.clone())
        g = torch.Generator().manual_seed(23)
        host, bs = [], []
        for _ in range(a.steps):
            u = torch.randint(0, U, (B,), generator=g).repeat_interleave(M)
            pick = torch.rand(B * M, generator=g) < 0.1
            u = torch.where(pick & (torch.arange(B * M) % M != 0),
                            torch.randint(0, U, (B * M,), generator=g), u)
            i = torch.randint(0, I, (B * M,), generator=g)
            t = torch.zeros(B, M)
            t[:, 0] = 1
            host.append((u.clone(), i.clone()))
            bs.append((copy(u.to(DEV)), copy(i.to(DEV)), copy(t.reshape(-1, 1).to(DEV))))
        torch.cuda.synchronize()
        for k, (u, i, _) in enumerate(bs):
            assert torch.equal(u.cpu(), host[k][0]) and torch.equal(i.cpu(), host[k][1]), k
        step = Tr.FusedTrainStep(m, lr=1e-3, weight_decay=1e-5)
        eng = m.engine
        for s, (u, i, t) in enumerate(bs):
            nxt = bs[s + 1][:2] if a.pipelined and s + 1 < len(bs) else None
            step(u, i, t, next=nxt)
            if a.sync_each:
                torch.cuda.synchronize()
                err = int(eng._err.item())
                bad = [k for k, (uu, ii, _) in enumerate(bs)
                       if not (torch.equal(uu.cpu(), host[k][0]) and torch.equal(ii.cpu(), host[k][1]))]
                w = next(iter(eng.ws.values()))
                nu = w.num_unique.cpu().tolist() if hasattr(w, "num_unique") else None
                uq = (w.uniq_u.cpu(), w.uniq_i.cpu())
                rng = None
                if nu is not None:
                    a0, a1 = int(nu[0]), int(nu[1])
                    rng = (int(uq[0][:a0].min()), int(uq[0][:a0].max()),
                           int(uq[1][:a1].min()), int(uq[1][:a1].max()))
                print(f"step {s}: err={err} corrupted_batches={bad} num_unique={nu} "
                      f"uniq_range={rng} expect=({len(set(host[s][0].tolist()))},"
                      f"{len(set(host[s][1].tolist()))})", flush=True)
                if err or bad:
                    for k in bad:
                        uu, ii, _ = bs[k]
                        du = (uu.cpu() != host[k][0]).nonzero().flatten()
                        di = (ii.cpu() != host[k][1]).nonzero().flatten()
                        print(f"  batch {k}: user ids differ at {du[:20].tolist()} "
                              f"(n={du.numel()}) got {uu.cpu()[du[:8]].tolist()}; item ids "
                              f"differ at {di[:20].tolist()} (n={di.numel()}) got "
                              f"{ii.cpu()[di[:8]].tolist()}", flush=True)
                    eng._err.zero_()
        step.sync()
        torch.cuda.synchronize()
        print("final err", int(eng._err.item()), flush=True)
        sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
        print("finite", all(torch.isfinite(v).all() for v in sd.values()), flush=True)
        del step, m
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
