"""Parity at the sizes the bench line is quoted on (BASELINE.json configs[1] / configs[4]).

* C2 (1M users x 100K items, D=64, H=4, MLP [256,128,64], B=4096 groups x M=5 = 20,480 rows,
  the bench's own Zipf(1.05) batches: 256 tower workgroups, 2-pass radix over 20-bit ids,
  multi-piece hot item segments): 3 training steps through ``FusedTrainStep`` (pipelined id
  sort, overlapped sweep, deferred dense-exact Adam) and 3 through the reference call pattern
  (``model(kjt)`` -> ``nn.BCELoss`` -> ``backward`` -> ``torch.optim.Adam.step``), each against
  ``oracle.train_step`` on the same initial weights and batches (dropout 0: our dropout masks
  are our own RNG).  Tolerances (tests/parity.py): probabilities abs 1e-6, loss
  abs 2e-6, every parameter of the model (all 1.1M table rows, touched or not) abs 1e-6 outside
  the per-step sign-flip zone, Adam moments at the F2 tolerances.
* C2 with bf16 tables: the same batches, loss within 1% of the fp32 oracle every step.
* C5 (10K users x 1M items, top-10 and top-100, ``GraphedScorer``): 64 sampled users against
  ``oracle.score_factorised`` over all 1M items: the same ids except between oracle scores tied
  within 1e-6, scores within 1e-6.

Reference: src/model/trainer.py:253-285, src/inference/demo/app.py:43-77."""
import numpy as np
import pytest
import torch

import _ncf_pkg
import bench
from oracle import ncf_oracle as O
from tests.parity import assert_moment_close, assert_params_close, zone_from_grads

pytestmark = pytest.mark.gpu
ncf = _ncf_pkg.load()
DEV = torch.device("cuda:0")

U, I, D, T, H, HID, B, M = 1_000_000, 100_000, 64, 32, 4, [256, 128, 64], 4096, 5
LR, WD, STEPS = 1e-3, 1e-5, 3


def _model(init):
    m = ncf.AdvancedNCF(U, I, 10, 50, D, D, T, HID, H, 0.0, M - 1)
    m.load_state_dict(init, strict=True)
    return m.to(DEV).train()


@pytest.fixture(scope="module")
def c2():
    """Initial weights, the bench's batches, and the oracle's 3-step trajectory."""
    torch.set_num_threads(bench.host_cpu()[0])
    torch.manual_seed(2024)
    m = ncf.AdvancedNCF(U, I, 10, 50, D, D, T, HID, H, 0.0, M - 1)
    init = {k: v.detach().clone() for k, v in m.state_dict().items()}
    del m
    batches = bench.make_batches(U, I, B, M, STEPS, DEV, seed=100)
    host = [(u.cpu(), i.cpu(), t.cpu()) for u, i, t in batches]
    ref = {k: v.clone() for k, v in init.items()}
    opt = O.AdamState(lr=LR, weight_decay=WD)
    probs, losses, zones = [], [], {}
    for u, i, t in host:
        before = {k: v.clone() for k, v in ref.items()}
        prob, loss, grads = O.train_step(ref, opt, u, i, t, negative_samples=M - 1, num_heads=H,
                                         temporal_dim=T, n_layers=len(HID))
        probs.append(prob.reshape(-1).numpy())
        losses.append(float(loss))
        for k, g in grads.items():
            zones.setdefault(k, []).append(zone_from_grads(g.numpy(), before[k].numpy(), WD))
        del before, grads
    uniq = [(int(u.unique().numel()), int(i.unique().numel())) for u, i, _ in host]
    # the case must hold what only full size has: hot item segments longer than one piece
    assert max(int(torch.bincount(i).max()) for _, i, _ in host) > 64
    return dict(init=init, batches=batches, probs=probs, losses=losses, ref=ref,
                state=opt.state, zones=zones, uniq=uniq)


def _check_params(c, sd, state):
    """Every parameter after STEPS steps vs the oracle (all rows of every table)."""
    for k, v in c["ref"].items():
        got = sd[k].detach().cpu().numpy()
        if k not in c["zones"]:          # unused by forward (grad None): never moves
            assert np.array_equal(got, c["init"][k].numpy()), k
            continue
        assert_params_close(k, got, v.numpy(), c["zones"][k], LR)
    for k, st in c["state"].items():
        zs = c["zones"][k]
        assert_moment_close(k, state[k]["exp_avg"], st["exp_avg"].numpy(), zs)
        assert_moment_close(k, state[k]["exp_avg_sq"], st["exp_avg_sq"].numpy(), zs, atol=1e-12)
        assert float(state[k]["step"]) == STEPS, k


def _check_step(c, s, prob, loss):
    d = np.abs(prob.reshape(-1) - c["probs"][s]).max()
    assert d <= 1e-6, f"step {s}: |dprob| {d:.3e}"
    assert abs(loss - c["losses"][s]) <= 2e-6, f"step {s}: loss {loss} vs {c['losses'][s]}"


def _torch_state(m, opt):
    names = {id(p): n for n, p in m.named_parameters()}
    return {names[id(p)]: {k: (v.detach().cpu().numpy() if torch.is_tensor(v) and v.dim() else
                               float(v)) for k, v in s.items()}
            for p, s in opt.state.items()}


def test_c2_full_size_fused_step_vs_oracle(c2):
    from ncf_amd.trainer import FusedTrainStep
    m = _model(c2["init"])
    step = FusedTrainStep(m, lr=LR, weight_decay=WD)
    bt = c2["batches"]
    for s, (u, i, t) in enumerate(bt):
        w = step(u, i, t, next=bt[s + 1][:2] if s + 1 < len(bt) else None)
        _check_step(c2, s, w.prob.detach().cpu().numpy(), float(w.loss.item()))
    assert tuple(w.num_unique.cpu().tolist()) == c2["uniq"][-1]   # (unique users, items)
    opt = torch.optim.Adam(m.parameters(), lr=LR, weight_decay=WD)
    step.export_optimizer_state(opt)
    _check_params(c2, m.state_dict(), _torch_state(m, opt))


def test_c2_full_size_reference_call_pattern_vs_oracle(c2):
    m = _model(c2["init"])
    opt = torch.optim.Adam(m.parameters(), lr=LR, weight_decay=WD)
    crit = torch.nn.BCELoss()
    for s, (u, i, t) in enumerate(c2["batches"]):
        kj = ncf.KeyedJaggedTensor.from_lengths_sync(
            keys=["user_id", "product_id"], values=torch.cat([u, i]),
            lengths=torch.ones(2 * u.numel(), dtype=torch.long, device=DEV))
        out = m(kj)
        loss = crit(out, t)
        opt.zero_grad()
        loss.backward()
        opt.step()
        _check_step(c2, s, out.detach().cpu().numpy(), float(loss.item()))
    _check_params(c2, m.state_dict(), _torch_state(m, opt))


def test_c2_full_size_bf16_tables_track_oracle(c2):
    from ncf_amd.trainer import FusedTrainStep
    m = _model(c2["init"])
    step = FusedTrainStep(m, lr=LR, weight_decay=WD, table_dtype=torch.bfloat16)
    for s, (u, i, t) in enumerate(c2["batches"]):
        w = step(u, i, t)
        rel = abs(float(w.loss.item()) - c2["losses"][s]) / c2["losses"][s]
        assert rel < 0.01, f"step {s}: bf16-table loss {rel:.3%} from the fp32 oracle"


# ----------------------------------------------------------------------------- C5
@pytest.mark.parametrize("k", [10, 100])
def test_c5_full_size_graphed_topk_vs_oracle(k, c5):
    from ncf_amd.scoring import GraphedScorer
    m, users, sel, ref, order = c5
    sc = GraphedScorer(m, users.numel(), k=k)
    s, it = sc(users.to(DEV))
    s, it = s[sel].cpu(), it[sel].cpu()
    for r in range(len(sel)):
        want = order[r, :k].tolist()
        got = it[r].tolist()
        if got != want:
            # identical ranking except where the oracle's own fp32 scores tie within 1e-6
            np.testing.assert_allclose(ref[r, got].numpy(), ref[r, want].numpy(), atol=1e-6)
        np.testing.assert_allclose(s[r].numpy(), ref[r, got].numpy(), atol=1e-6)


@pytest.fixture(scope="module")
def c5():
    torch.set_num_threads(bench.host_cpu()[0])
    torch.manual_seed(4321)
    NU, NI = 1_000_000, 1_000_000
    m = ncf.AdvancedNCF(NU, NI, 10, 50).to(DEV).eval()
    users = torch.randperm(NU)[:10_000]
    sel = torch.randperm(users.numel(), generator=torch.Generator().manual_seed(5))[:64]
    p = {kk: v.detach().cpu() for kk, v in m.state_dict().items()}
    with torch.no_grad():
        ref = O.score_factorised(p, users[sel], torch.arange(NI), temporal_dim=32, n_layers=3)
    order = torch.stack([torch.argsort(-ref[r], stable=True)[:100] for r in range(len(sel))])
    return m, users, sel, ref, order
