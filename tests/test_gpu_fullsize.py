"""Parity at the sizes the bench line is quoted on (BASELINE.json configs[1] / configs[4]).

* C2 (1M users x 100K items, D=64, H=4, MLP [256,128,64], B=4096 groups x M=5 = 20,480 rows,
  the bench's own Zipf(1.05) batches: 256 tower workgroups, 2-pass radix over 20-bit ids,
  multi-piece hot item segments): 3 training steps through ``FusedTrainStep`` (pipelined id
  sort, overlapped sweep, deferred dense-exact Adam) and 3 through the reference call pattern
  (``model(kjt)`` -> ``nn.BCELoss`` -> ``backward`` -> ``torch.optim.Adam.step``), each against
  ``oracle.train_step`` on the same initial weights and batches (dropout 0: our dropout masks
  are our own RNG).  The oracle runs twice, in fp32 (the reference's precision) and in fp64
  (the exact trajectory).  Tolerances (tests/parity.py): step 0's probabilities
  abs 1e-6 from the fp32 oracle, loss abs 2e-6; every parameter of the model (all 1.1M table
  rows, touched or not) abs 1e-6 from the exact trajectory outside the per-step sign-flip zone.
  At this size the fp32 oracle is itself far off the exact trajectory after the first Adam
  step: Adam (eps 1e-8) turns fp32 rounding noise in near-zero gradients into +-lr steps that
  the fp64 run does not take (measured on the MI355X box's host: step-1 / step-2 probabilities
  3.1e-5 / 1.9e-3 off, ~20K item-table elements outside the exact zone up to 4.3e-3 off).  So
  later steps and those elements are held to the fp32 oracle's own distance from the exact
  trajectory (x4; the GPU measured within 1% of it in count and worst case), and the elements of
  the fp32 oracle's own sign-flip zone to 2 lr per zone step from it.  On top of that every
  step's probabilities and every parameter are held directly to the fp32 oracle at what was
  measured: probabilities 2e-5, per table <= 400 elements outside its zone off by > 1e-6 (each
  <= 2e-4), dense parameters 1e-5 (_check_step / _check_params; per-tensor numbers written to
  gpurun_out/fullsize_*.json).
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
from tests.parity import zone_from_grads

pytestmark = pytest.mark.gpu
ncf = _ncf_pkg.load()
DEV = torch.device("cuda:0")

U, I, D, T, H, HID, B, M = 1_000_000, 100_000, 64, 32, 4, [256, 128, 64], 4096, 5
LR, WD, STEPS = 1e-3, 1e-5, 3
ATOL = 1e-6
# Direct bounds against the fp32 oracle (the reference's own precision), outside its own
# sign-flip zone, set at the measured distances with headroom:
PROB_FP32 = 2e-5              # steps >= 1 (measured 3.1e-6 / 1.06e-5 at steps 1 / 2)
TABLE_OFF, TABLE_OFF_MAX = 400, 2e-4     # per table (measured 74-139 elements, <= 8.8e-5)
DENSE_OFF_MAX = 1e-5          # every dense element (measured 3.1e-6)
TABLES = {f"{p}_embedding_collection.embedding_bags.{t}.weight" for p in ("mf", "mlp")
          for t in ("user_id", "product_id")}


def _model(init):
    m = ncf.AdvancedNCF(U, I, 10, 50, D, D, T, HID, H, 0.0, M - 1)
    m.load_state_dict(init, strict=True)
    return m.to(DEV).train()


@pytest.fixture(scope="module")
def c2():
    """Initial weights, the bench's batches, and the oracle's 3-step trajectory twice: in fp32
    (the reference's precision) and in fp64 (the exact trajectory both fp32 computations are
    measured against)."""
    torch.set_num_threads(bench.host_cpu()[0])
    torch.manual_seed(2024)
    m = ncf.AdvancedNCF(U, I, 10, 50, D, D, T, HID, H, 0.0, M - 1)
    init = {k: v.detach().clone() for k, v in m.state_dict().items()}
    del m
    batches = bench.make_batches(U, I, B, M, STEPS, DEV, seed=100)
    host = [(u.cpu(), i.cpu(), t.cpu()) for u, i, t in batches]
    out = dict(init=init, batches=batches)
    zones = {}
    for tag, dt in (("o32", torch.float32), ("o64", torch.float64)):
        ref = {k: v.to(dt).clone() for k, v in init.items()}
        opt = O.AdamState(lr=LR, weight_decay=WD)
        probs, losses = [], []
        zt = zones.setdefault(tag, {})
        for u, i, t in host:
            before = {k: v.numpy().copy() for k, v in ref.items()}
            prob, loss, grads = O.train_step(ref, opt, u, i, t.to(dt), negative_samples=M - 1,
                                             num_heads=H, temporal_dim=T, n_layers=len(HID))
            probs.append(prob.reshape(-1).double().numpy())
            losses.append(float(loss))
            for k, g in grads.items():   # each step's sign-flip zone, from each run's gradients
                zt.setdefault(k, []).append(zone_from_grads(g.numpy(), before[k], WD))
            del before, grads
        out[tag] = dict(probs=probs, losses=losses, ref=ref, state=opt.state)
    out["zones"] = zones["o64"]
    out["zones32"] = zones["o32"]
    # the case must hold what only full size has: hot item segments longer than one piece
    assert max(int(torch.bincount(i).max()) for _, i, _ in host) > 64
    out["uniq"] = [(int(u.unique().numel()), int(i.unique().numel())) for u, i, _ in host]
    # the fp32 reference's own distance from the exact trajectory (the noise floor of any fp32
    # implementation at this size): per tensor, elements outside the zone off by > 1e-6
    out["noise"] = {k: _dev(out["o32"]["ref"][k].double().numpy(), out["o64"]["ref"][k].numpy(),
                            z) for k, z in out["zones"].items()}
    return out


def _dev(a, exact, zones):
    """(count, max) of |a - exact| > ATOL outside the sign-flip zone, and (count, max) inside."""
    d = np.abs(np.asarray(a, np.float64) - exact)
    nz = np.sum(zones, axis=0)
    bad = d > ATOL
    o, z = bad & (nz == 0), bad & (nz > 0)
    return (int(o.sum()), float(d[o].max()) if o.any() else 0.0,
            int(z.sum()), float(d[z].max()) if z.any() else 0.0)


def _stats(name, rec):
    """Write the measured deviations next to the gpu run's outputs (evidence for DESIGN.md)."""
    import json
    import os
    d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    if os.path.isdir(d):
        with open(os.path.join(d, f"fullsize_{name}.json"), "w") as f:
            json.dump(rec, f, indent=1)


def _check_params(c, sd, state, name, rec):
    """Every parameter after STEPS steps against the exact (fp64) trajectory.  Outside the
    (exact) sign-flip zone an element is within ATOL, except for as many elements as the fp32 oracle
    itself misses there (x4, + 16), each within max(4 x the oracle's own worst, 1e-5); inside
    the fp32 reference's own zone within 2 lr per zone step of it (tests/parity.py; the exact
    trajectory does not take those noise-driven steps at all).  Adam moments outside the zone within
    max(4 x the fp32 oracle's own worst, 1e-7 / 1e-12).  Unused parameters never move."""
    lr_bound = 2 * LR
    fails = []
    rec["params"] = {}
    for k, v in c["o64"]["ref"].items():
        got = sd[k].detach().cpu().numpy()
        if k not in c["zones"]:          # unused by forward (grad None): never moves
            if not np.array_equal(got, c["init"][k].numpy()):
                fails.append(f"{k}: unused parameter moved")
            continue
        zs = c["zones"][k]
        n_o, m_o, n_z, m_z = _dev(got, v.numpy(), zs)
        nn_o, nm_o = c["noise"][k][:2]
        rec["params"][k] = {"gpu_vs_fp64": [n_o, m_o, n_z, m_z], "fp32_oracle_vs_fp64":
                            list(c["noise"][k])}
        if n_o > 4 * nn_o + 16 or m_o > max(4 * nm_o, 1e-5):
            fails.append(f"{k}: {n_o} elements outside the zone off by up to {m_o:.3e} "
                         f"(fp32 oracle: {nn_o}, {nm_o:.3e})")
        # against the fp32 reference itself (the F2 rule, tests/parity.py): inside its own
        # sign-flip zone an element is within 2 lr per zone step
        z32 = c["zones32"][k]
        nz32 = np.sum(z32, axis=0)
        d32 = np.abs(got - c["o32"]["ref"][k].numpy())
        rec["params"][k]["gpu_vs_fp32"] = list(_dev(got, c["o32"]["ref"][k].double().numpy(), z32))
        if ((nz32 > 0) & (d32 > lr_bound * nz32 + ATOL)).any():
            fails.append(f"{k}: fp32-zone element beyond 2 lr per zone step")
        # ... and outside it, bound at what was measured (round 4: <= 139 table elements off by
        # <= 8.8e-5, dense <= 3.1e-6; a 10x regression fails): tables at most TABLE_OFF elements
        # off by > ATOL, each <= TABLE_OFF_MAX; dense parameters every element <= DENSE_OFF_MAX
        n32, m32 = rec["params"][k]["gpu_vs_fp32"][:2]
        if k in TABLES:
            if n32 > TABLE_OFF or m32 > TABLE_OFF_MAX:
                fails.append(f"{k}: {n32} elements outside the fp32 zone off the fp32 oracle by "
                             f"up to {m32:.3e} (bound {TABLE_OFF}, {TABLE_OFF_MAX:.0e})")
        elif m32 > DENSE_OFF_MAX:
            fails.append(f"{k}: {m32:.3e} off the fp32 oracle outside its zone "
                         f"(bound {DENSE_OFF_MAX:.0e})")
    rec["moments"] = {}
    for k, st in c["o64"]["state"].items():
        zone = np.any(c["zones"][k], axis=0)
        for mom, atol in (("exp_avg", 1e-7), ("exp_avg_sq", 1e-12)):
            exact = st[mom].numpy()
            g = np.abs(np.asarray(state[k][mom], np.float64) - exact)[~zone]
            o = np.abs(c["o32"]["state"][k][mom].double().numpy() - exact)[~zone]
            gm, om = (float(g.max()) if g.size else 0.0), (float(o.max()) if o.size else 0.0)
            rec["moments"][f"{k}.{mom}"] = [gm, om]
            if gm > max(4 * om, atol):
                fails.append(f"{k}.{mom}: {gm:.3e} off outside the zone (fp32 oracle {om:.3e})")
        if float(state[k]["step"]) != STEPS:
            fails.append(f"{k}: step {state[k]['step']}")
    _stats(name, rec)
    assert not fails, "; ".join(fails[:8])


def _check_step(c, s, prob, loss, rec):
    """Step s's probabilities and loss.  Step 0 runs on the initial weights: abs 1e-6 from the
    fp32 oracle.  Every step: within max(4 x the fp32 oracle's own distance from the exact
    (fp64) probabilities, 2e-6) of them — after the first Adam step the sign-flip zone's
    elements (|g + wd p| < 1e-6, moved +-lr by summation noise) put both fp32 computations
    1e-6..1e-5 off the exact trajectory at this size.  Loss: abs 2e-6 from the fp32 oracle."""
    p = prob.reshape(-1).astype(np.float64)
    d32 = float(np.abs(p - c["o32"]["probs"][s]).max())
    d64 = float(np.abs(p - c["o64"]["probs"][s]).max())
    n64 = float(np.abs(c["o32"]["probs"][s] - c["o64"]["probs"][s]).max())
    dl = abs(loss - c["o32"]["losses"][s])
    rec.setdefault("steps", []).append({"dprob_vs_fp32": d32, "dprob_vs_fp64": d64,
                                        "fp32_oracle_dprob_vs_fp64": n64, "dloss_vs_fp32": dl})
    if s == 0:
        assert d32 <= 1e-6, f"step 0: |dprob| {d32:.3e} from the fp32 oracle"
    assert d32 <= PROB_FP32, f"step {s}: |dprob| {d32:.3e} from the fp32 oracle"
    assert d64 <= max(4 * n64, 2e-6), f"step {s}: |dprob| {d64:.3e} vs fp64 (fp32 oracle {n64:.3e})"
    assert dl <= 2e-6, f"step {s}: loss {loss} vs {c['o32']['losses'][s]}"


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
    rec = {}
    for s, (u, i, t) in enumerate(bt):
        w = step(u, i, t, next=bt[s + 1][:2] if s + 1 < len(bt) else None)
        _check_step(c2, s, w.prob.detach().cpu().numpy(), float(w.loss.item()), rec)
    assert tuple(w.num_unique.cpu().tolist()) == c2["uniq"][-1]   # (unique users, items)
    opt = torch.optim.Adam(m.parameters(), lr=LR, weight_decay=WD)
    step.export_optimizer_state(opt)
    _check_params(c2, m.state_dict(), _torch_state(m, opt), "fused", rec)


def test_c2_full_size_reference_call_pattern_vs_oracle(c2):
    m = _model(c2["init"])
    opt = torch.optim.Adam(m.parameters(), lr=LR, weight_decay=WD)
    crit = torch.nn.BCELoss()
    rec = {}
    for s, (u, i, t) in enumerate(c2["batches"]):
        kj = ncf.KeyedJaggedTensor.from_lengths_sync(
            keys=["user_id", "product_id"], values=torch.cat([u, i]),
            lengths=torch.ones(2 * u.numel(), dtype=torch.long, device=DEV))
        out = m(kj)
        loss = crit(out, t)
        opt.zero_grad()
        loss.backward()
        opt.step()
        _check_step(c2, s, out.detach().cpu().numpy(), float(loss.item()), rec)
    _check_params(c2, m.state_dict(), _torch_state(m, opt), "dropin", rec)


def test_c2_full_size_bf16_tables_track_oracle(c2):
    from ncf_amd.trainer import FusedTrainStep
    m = _model(c2["init"])
    step = FusedTrainStep(m, lr=LR, weight_decay=WD, table_dtype=torch.bfloat16)
    for s, (u, i, t) in enumerate(c2["batches"]):
        w = step(u, i, t)
        rel = abs(float(w.loss.item()) - c2["o32"]["losses"][s]) / c2["o32"]["losses"][s]
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
