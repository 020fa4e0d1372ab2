"""Find a buffer that a training step reads before anything writes it (GPU only).

The guarded fused step (tests/test_gpu_guard.py) is run once with its allocations left as the
guard arena makes them, then with every uninitialised allocation poisoned (NaN floats, integer
1: tests/guard_alloc.py), and the final parameters, moments and engine flag compared bit for bit.
If poisoning changes them, some kernel read a buffer before writing it (a result that depends on
what the memory held before: the process history); the allocation sites are then bisected
(poison one half, compare) down to one site.

    python tools/guard_bisect.py [--fuse-apply 0|1] [--early-reduce 0|1] [--pipelined 0|1]
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


def run(cfg, poison, steps=6):
    """-> (state dict + moments on the host, engine id flag after the run)."""
    import ncf_amd.trainer as Tr
    from ncf_amd import engine as E
    Tr.FUSE_APPLY, Tr.EARLY_REDUCE = bool(cfg.fuse_apply), bool(cfg.early_reduce)
    E.GROUP_ROWS = True
    U, I, B, M = 3000, 500, 61, 5
    torch.manual_seed(24)
    m = ncf.AdvancedNCF(U, I, 5, 24, 64, 64, 32, [256, 128, 64], 4, 0.2, M - 1).to(DEV)
    with guarded(poison=poison) as arena:
        g = torch.Generator().manual_seed(23)
        bs = []
        for _ in range(steps):
            u = torch.randint(0, U, (B,), generator=g).repeat_interleave(M)
            pick = torch.rand(B * M, generator=g) < 0.1
            u = torch.where(pick & (torch.arange(B * M) % M != 0),
                            torch.randint(0, U, (B * M,), generator=g), u)
            i = torch.randint(0, I, (B * M,), generator=g)
            t = torch.zeros(B, M)
            t[:, 0] = 1
            bs.append((arena.copy(u.to(DEV)), arena.copy(i.to(DEV)),
                       arena.copy(t.reshape(-1, 1).to(DEV))))
        step = Tr.FusedTrainStep(m, lr=1e-3, weight_decay=1e-5)
        flags = torch.zeros(steps, dtype=torch.int32).pin_memory()
        for s, (u, i, t) in enumerate(bs):
            nxt = bs[s + 1][:2] if cfg.pipelined and s + 1 < len(bs) else None
            step(u, i, t, next=nxt)
            flags[s:s + 1].copy_(m.engine._err, non_blocking=True)   # (no host sync)
        step.sync()
        torch.cuda.synchronize()
        eng = m.engine
        err = int(eng._err.item())
        if err:
            print(f"    id flag per step: {flags.tolist()}", flush=True)
        eng._err.zero_()
        eng._err_async = None
        sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
        mom = {k: (v["exp_avg"].cpu().clone(), v["exp_avg_sq"].cpu().clone())
               for k, v in step.state.items()}
        del step, m
        torch.cuda.synchronize()
    return sd, mom, err


def same(a, b):
    sa, ma, ea = a
    sb, mb, eb = b
    bad = [k for k in sa if not torch.equal(sa[k], sb[k])]
    bad += [k + ".m" for k in ma if not (torch.equal(ma[k][0], mb[k][0]) and
                                         torch.equal(ma[k][1], mb[k][1]))]
    return (not bad and ea == eb), bad, (ea, eb)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fuse-apply", type=int, default=0)
    ap.add_argument("--early-reduce", type=int, default=0)
    ap.add_argument("--pipelined", type=int, default=0)
    cfg = ap.parse_args()
    sites = []

    def collect(site):
        if site not in sites:
            sites.append(site)
        return False
    base = run(cfg, collect)
    again = run(cfg, False)
    ok, bad, errs = same(base, again)
    print(f"config {vars(cfg)}: {len(sites)} allocation sites; unpoisoned rerun same: {ok} "
          f"{bad[:5]} err {errs}", flush=True)
    full = run(cfg, True)
    ok, bad, errs = same(base, full)
    print(f"all poisoned: same {ok}; differing {len(bad)}: {bad[:8]} err {errs}", flush=True)
    if ok:
        return
    cand = list(sites)
    while len(cand) > 1:
        half = cand[:len(cand) // 2]
        hs = set(half)
        ok, bad, errs = same(base, run(cfg, lambda s, hs=hs: s in hs))
        print(f"  poison {len(half)} of {len(cand)} sites: same {ok} ({len(bad)} differ, err "
              f"{errs})", flush=True)
        if not ok:
            cand = half
            continue
        rest = cand[len(cand) // 2:]
        rs = set(rest)
        ok2, bad2, errs2 = same(base, run(cfg, lambda s, rs=rs: s in rs))
        print(f"  poison the other {len(rest)}: same {ok2} ({len(bad2)} differ, err {errs2})",
              flush=True)
        if ok2:
            print("  neither half alone changes the result: it takes sites from both", flush=True)
            print("  remaining:", cand, flush=True)
            return
        cand = rest
    print("READ BEFORE WRITE at allocation site:", cand, flush=True)


if __name__ == "__main__":
    main()
