"""Out-of-bounds read audit of the ragged training / scoring paths (marker ``gpu``).

Every CUDA buffer the package allocates while these tests run — workspaces, dedup sets, the
deferred Adam's stamps and scalar table, the reduction scratch, the scoring buffers — and every
input id / target tensor sits at the END of its own mapping with unmapped address space behind
it (tests/guard_alloc.py).  A kernel that reads more than 16 bytes past the end of any of them
(the padded rows of a ragged last workgroup, a prefetch one tile too far) faults in the launch
that made the read, instead of reading a neighbour's bytes as it does under the caching
allocator.  Batch sizes are chosen so that every tiled kernel has a ragged last workgroup (61
groups of 5: 3 full 16-group attention/tower tiles + 13 groups).

The r05y fault (What's weak 1) surfaced once in `test_group_rows_bitwise_equals_
every_row[True]` with a library that passed the same test in another process: a read past the
end of a buffer that only faults when the allocation history leaves that buffer at the end of a
mapped segment is the one mechanism that depends on what ran before in the process.  These
tests pin that no such read exists on the paths that test drives, in every configuration of the
schedule switches it could have run with (trainer.FUSE_APPLY, trainer.EARLY_REDUCE).
"""
import gc
import os

import pytest
import torch

import _ncf_pkg
from tests.guard_alloc import guarded

pytestmark = pytest.mark.gpu
ncf = _ncf_pkg.load()
DEV = torch.device("cuda:0")
LOG = os.environ.get("NCF_GUARD_LOG")     # (fault triage: the arena's address map)


def _batches(arena, U, I, B, M, steps, mixed, seed=23):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(steps):
        u = torch.randint(0, U, (B,), generator=g).repeat_interleave(M)
        if mixed:
            pick = torch.rand(B * M, generator=g) < 0.1
            u = torch.where(pick & (torch.arange(B * M) % M != 0),
                            torch.randint(0, U, (B * M,), generator=g), u)
        i = torch.randint(0, I, (B * M,), generator=g)
        t = torch.zeros(B, M)
        t[:, 0] = 1
        out.append((arena.copy(u.to(DEV)), arena.copy(i.to(DEV)),
                    arena.copy(t.reshape(-1, 1).to(DEV))))
    return out


def _drop(*_objs):
    """Drain the device before the arena unmaps what these objects' buffers live in."""
    gc.collect()
    torch.cuda.synchronize()


@pytest.mark.parametrize("fuse_apply", [True, False])
@pytest.mark.parametrize("early_reduce", [False, True])
@pytest.mark.parametrize("pipelined", [False, True])
def test_guarded_fused_step_mixed_groups_ragged(monkeypatch, fuse_apply, early_reduce, pipelined):
    """The r05y configuration (mixed user ids inside groups, group rows on, the fused attention
    + tower, 61 groups) under guard pages, over the schedule switches; then the state_dict read
    that surfaced the fault."""
    import ncf_amd.trainer as Tr
    from ncf_amd import engine as E
    monkeypatch.setattr(Tr, "FUSE_APPLY", fuse_apply)
    monkeypatch.setattr(Tr, "EARLY_REDUCE", early_reduce)
    monkeypatch.setattr(E, "GROUP_ROWS", True)
    U, I, B, M = 3000, 500, 61, 5
    torch.manual_seed(24)
    m = ncf.AdvancedNCF(U, I, 5, 24, 64, 64, 32, [256, 128, 64], 4, 0.2, M - 1).to(DEV)
    with guarded(log=LOG) as arena:
        step = Tr.FusedTrainStep(m, lr=1e-3, weight_decay=1e-5)
        bs = _batches(arena, U, I, B, M, 6, mixed=True)
        for s, (u, i, t) in enumerate(bs):
            nxt = bs[s + 1][:2] if pipelined and s + 1 < len(bs) else None
            step(u, i, t, next=nxt)
        assert next(iter(m.engine.ws.values())).group_rows == M
        step.sync()
        sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
        assert all(torch.isfinite(v).all() for v in sd.values())
        assert arena.count > 50
        _drop(step, m, bs)


def test_guarded_reference_call_pattern_ragged():
    """model(kjt) -> BCELoss -> backward -> torch.optim.Adam.step (the drop-in hook: claim-path
    catch-up, the id sort forked beside the forward, launch tapes from the third step) with a
    ragged batch, then an eval forward of a ragged row count."""
    U, I, B, M = 2000, 300, 61, 5
    torch.manual_seed(5)
    m = ncf.AdvancedNCF(U, I, 5, 24, 64, 64, 32, [256, 128, 64], 4, 0.2, M - 1).to(DEV)
    with guarded(log=LOG) as arena:
        opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-5)
        crit = torch.nn.BCELoss()
        m.train()
        for u, i, t in _batches(arena, U, I, B, M, 5, mixed=True, seed=3):
            kjt = ncf.KeyedJaggedTensor.from_lengths_sync(
                keys=["user_id", "product_id"], values=arena.copy(torch.cat([u, i])),
                lengths=arena.copy(torch.ones(2 * u.numel(), dtype=torch.long, device=DEV)))
            loss = crit(m(kjt), t)
            opt.zero_grad()
            loss.backward()
            opt.step()
        m.eval()
        g = torch.Generator().manual_seed(9)
        u = arena.copy(torch.randint(0, U, (77,), generator=g).to(DEV))
        i = arena.copy(torch.randint(0, I, (77,), generator=g).to(DEV))
        with torch.no_grad():
            p = m.forward_simple(u, i)
        assert torch.isfinite(p).all()
        _drop(opt, m, p)


@pytest.mark.parametrize("dims", ["c1", "c4", "bf16"])
def test_guarded_other_geometries_ragged(dims):
    """The unfused path at C1 dims (D = 16, H = 1, MLP [64, 32]), the D = 128 (C4) attention
    block, and the bf16-table configuration, each with a ragged batch."""
    from ncf_amd.trainer import FusedTrainStep
    if dims == "c1":
        args, B, M = (800, 400, 5, 24, 16, 16, 32, [64, 32], 1, 0.2, 4), 37, 5
    elif dims == "c4":
        args, B, M = (900, 300, 5, 24, 128, 128, 32, [256, 128, 64], 4, 0.2, 4), 21, 5
    else:
        args, B, M = (900, 300, 5, 24, 64, 64, 32, [256, 128, 64], 4, 0.2, 4), 61, 5
    torch.manual_seed(2)
    m = ncf.AdvancedNCF(*args).to(DEV)
    with guarded(log=LOG) as arena:
        kw = {"table_dtype": torch.bfloat16} if dims == "bf16" else {}
        step = FusedTrainStep(m, lr=1e-3, weight_decay=1e-5, **kw)
        for u, i, t in _batches(arena, args[0], args[1], B, M, 4, mixed=False, seed=4):
            step(u, i, t)
        step.sync()
        assert all(torch.isfinite(v).all() for v in m.state_dict().values())
        _drop(step, m)


def test_guarded_scoring_ragged():
    """C5 top-K (threshold sample, MFMA collect, select) for a ragged user count against a
    catalogue that is not a multiple of any tile."""
    from ncf_amd.scoring import score_topk
    torch.manual_seed(3)
    m = ncf.AdvancedNCF(700, 5003, 5, 24, 64, 64, 32, [256, 128, 64], 4, 0.0, 4).to(DEV).eval()
    with guarded(log=LOG) as arena:
        users = arena.copy(torch.randint(0, 700, (45,)).to(DEV))
        s, it = score_topk(m, users, k=10)
        s2, it2 = score_topk(m, users, k=100)
        torch.cuda.synchronize()
        assert torch.isfinite(s).all() and torch.isfinite(s2).all()
        _drop(m, s, it, s2, it2)
