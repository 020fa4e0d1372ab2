"""The reference call pattern on the fused path (src/model/trainer.py:258-285: ``model(kjt)`` ->
``nn.BCELoss`` -> ``zero_grad`` -> ``backward`` -> ``torch.optim.Adam.step``), and everything
that reads the tables while a deferred dense-exact schedule holds rows behind.  MI355X only.

Equalities here are bitwise: the deferred schedule replays every zero-gradient step with the
arithmetic and per-step scalars of the dense sweep, so the two must agree to the bit."""
import numpy as np
import pytest
import torch

import _ncf_pkg

pytestmark = pytest.mark.gpu
ncf = _ncf_pkg.load()
DEV = torch.device("cuda:0")
U, I, B, M = 3000, 500, 64, 5


def kjt(u, i):
    return ncf.KeyedJaggedTensor.from_lengths_sync(
        keys=["user_id", "product_id"], values=torch.cat([u, i]),
        lengths=torch.ones(2 * u.numel(), dtype=torch.long, device=u.device))


def batches(n, seed=5):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        u = torch.randint(0, U, (B,), generator=g).repeat_interleave(M).to(DEV)
        i = torch.randint(0, I, (B * M,), generator=g).to(DEV)
        t = torch.zeros(B, M)
        t[:, 0] = 1
        out.append((u, i, t.reshape(-1, 1).to(DEV)))
    return out


def model(dropout=0.0, seed=11):
    torch.manual_seed(seed)
    return ncf.AdvancedNCF(U, I, 5, 24, 64, 64, 32, [256, 128, 64], 4, dropout, M - 1).to(DEV)


def reference_loop(m, opt, data, lr_at=None):
    """trainer.py:258-285 (no clipping: the reference's guard is always False)."""
    crit = torch.nn.BCELoss()
    m.train()
    for s, (u, i, t) in enumerate(data):
        if lr_at and s in lr_at:
            for g in opt.param_groups:
                g["lr"] = lr_at[s]
        out = m(kjt(u, i))
        loss = crit(out, t)
        opt.zero_grad()
        loss.backward()
        opt.step()
    return loss


def snapshot(m, opt):
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    st = opt.state_dict()["state"]
    mom = {k: {n: (v.cpu().clone() if torch.is_tensor(v) else v) for n, v in s.items()}
           for k, s in st.items()}
    return sd, mom


def assert_same(a, b):
    for k in a[0]:
        assert torch.equal(a[0][k], b[0][k]), k
    assert set(a[1]) == set(b[1])
    for k in a[1]:
        for n in ("exp_avg", "exp_avg_sq", "step"):
            assert torch.equal(a[1][k][n], b[1][k][n]), (k, n)


def run_schedule(schedule, data, monkeypatch, lr_at=None):
    from ncf_amd import optim
    monkeypatch.setattr(optim, "SCHEDULE", schedule)
    m = model()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-5)
    reference_loop(m, opt, data, lr_at)
    return snapshot(m, opt), m, opt


@pytest.mark.parametrize("every,steps", [(64, 70), (128, 140)])
def test_hooked_deferred_bitwise_equals_dense_hook(monkeypatch, every, steps):
    """torch.optim.Adam.step() through the hook: the deferred schedule (catch-up in the
    forward, apply + 1/every sweep in the step) == the dense per-step table sweep, bit for bit,
    crossing a full sweep cycle (128: optim.SWEEP_EVERY's default), params and the optimizer's
    torch-format state."""
    from ncf_amd import optim as O
    monkeypatch.setattr(O, "SWEEP_EVERY", every)
    data = batches(steps)
    a, _, _ = run_schedule("dense", data, monkeypatch)
    b, m, opt = run_schedule("deferred", data, monkeypatch)
    assert_same(a, b)
    from ncf_amd import optim
    assert optim.binding_of(opt, m).D is not None     # the deferred path really ran


def test_launch_tapes_bitwise_equal_eager(monkeypatch):
    """The reference loop with its phases replayed from launch tapes (tapes.py) == the eager
    host code, bit for bit: dropout on, an lr change (scalar table refilled in place), a
    betas change (tapes dropped and recorded again), an eval forward and a state_dict read
    between steps (rows swept: the next backward / step run eagerly), gradient accumulation
    and a short last batch (another geometry)."""
    from ncf_amd import tapes
    data = batches(30, seed=31)
    short = batches(2, seed=32)
    crit = torch.nn.BCELoss()

    def run(enabled):
        monkeypatch.setattr(tapes, "ENABLED", enabled)
        m = model(dropout=0.2, seed=33)
        opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-5)
        losses = []
        m.train()
        for s, (u, i, t) in enumerate(data):
            if s == 11:
                for g in opt.param_groups:
                    g["lr"] = 2e-3
            if s == 19:
                for g in opt.param_groups:
                    g["betas"] = (0.85, 0.995)
            if s == 15:
                m.eval()
                with torch.no_grad():
                    m(kjt(u[:10], i[:10]))
                m.train()
            if s == 17:
                m.state_dict()
            out = m(kjt(u, i))
            loss = crit(out, t)
            opt.zero_grad()
            loss.backward()
            if s == 23:          # accumulate a second batch into this step
                crit(m(kjt(*short[0][:2])), short[0][2]).backward()
            opt.step()
            losses.append(loss.detach())
        su, si, st_ = short[1]
        crit(m(kjt(su[:160], si[:160])), st_[:160]).backward()
        opt.step()
        return snapshot(m, opt), torch.stack(losses).cpu(), m
    a, la, _ = run(False)
    b, lb, m = run(True)
    assert torch.equal(la, lb)
    assert_same(a, b)
    assert m.engine.tapes.replays > 20, m.engine.tapes.replays


def test_hooked_lr_change_bitwise_equals_dense_hook(monkeypatch):
    """An lr change mid-run (a scheduler) applies to the steps not yet taken; rows still behind
    replay the earlier steps with the lr those steps had."""
    data = batches(40, seed=8)
    lr_at = {13: 3e-3, 29: 5e-4}
    a, _, _ = run_schedule("dense", data, monkeypatch, lr_at)
    b, _, _ = run_schedule("deferred", data, monkeypatch, lr_at)
    assert_same(a, b)


def test_hooked_state_dict_roundtrip_resumes_exactly(monkeypatch):
    """opt.state_dict() / model.state_dict() mid-run (rows current first), loaded into a fresh
    model + torch Adam, then continued == the uninterrupted run."""
    data = batches(30, seed=9)
    whole, _, _ = run_schedule("deferred", data, monkeypatch)
    m1 = model()
    o1 = torch.optim.Adam(m1.parameters(), lr=1e-3, weight_decay=1e-5)
    reference_loop(m1, o1, data[:17])
    msd = {k: v.clone() for k, v in m1.state_dict().items()}
    osd = o1.state_dict()
    m2 = model(seed=99)
    o2 = torch.optim.Adam(m2.parameters(), lr=1e-3, weight_decay=1e-5)
    m2.load_state_dict(msd)
    o2.load_state_dict(osd)
    reference_loop(m2, o2, data[17:])
    assert_same(whole, snapshot(m2, o2))


def test_load_state_dict_mid_run_does_not_replay_old_steps(tmp_path):
    """a checkpoint loaded into a model whose deferred schedule still owes rows
    zero-gradient steps must not get those steps replayed onto the loaded rows.  Train 12 steps,
    load the step-5 checkpoint into the same model + step, continue: == a fresh model resumed
    from the same checkpoint."""
    from ncf_amd.checkpoint import load_checkpoint, save_checkpoint
    from ncf_amd.trainer import FusedTrainStep
    data = batches(20, seed=12)

    def fresh():
        m = model(seed=4)
        return m, FusedTrainStep(m, lr=1e-2, weight_decay=1e-5)
    m1, s1 = fresh()
    for b in data[:5]:
        s1(*b)
    path = str(tmp_path / "ck.pt")
    save_checkpoint(path, m1, s1, epoch=0)
    for b in data[5:12]:
        s1(*b)
    load_checkpoint(path, m1, s1)          # rows of steps 6..12 still lag here
    for b in data[12:]:
        s1(*b)
    m2, s2 = fresh()
    load_checkpoint(path, m2, s2)
    for b in data[12:]:
        s2(*b)
    a, b_ = m1.state_dict(), m2.state_dict()
    for k in a:
        assert torch.equal(a[k], b_[k]), k


def test_direct_table_readers_see_current_rows():
    """after FusedTrainSteps on the deferred schedule, every direct read of the
    tables — the collection's forward (app.py:156 ``model.mlp_embedding_collection(kjt)``), a
    bag's ``.weight``, a submodule's state_dict — equals the dense schedule's rows bitwise."""
    from ncf_amd.trainer import FusedTrainStep
    data = batches(10, seed=13)
    res = []
    for deferred in (False, True):
        m = model(seed=21)
        step = FusedTrainStep(m, lr=1e-3, weight_decay=1e-5, deferred=deferred)
        for b in data:
            step(*b)
        ids = torch.arange(0, U, 7, device=DEV)
        feats = kjt(ids, ids % I)
        coll = m.mlp_embedding_collection(feats)
        if deferred:
            assert not m.engine.lagging()          # the read above brought every row current
        w = m.mf_embedding_collection.embedding_bags["product_id"].weight.detach().clone()
        sub = m.mlp_embedding_collection.state_dict()
        res.append((coll["user_id"].cpu(), coll["product_id"].cpu(), w.cpu(),
                    {k: v.cpu().clone() for k, v in sub.items()}))
    for x, y in zip(res[0][:3], res[1][:3]):
        assert torch.equal(x, y)
    for k in res[0][3]:
        assert torch.equal(res[0][3][k], res[1][3][k]), k


def test_bag_weight_read_syncs_lagging_rows():
    from ncf_amd.trainer import FusedTrainStep
    m = model(seed=22)
    step = FusedTrainStep(m, lr=1e-3, weight_decay=1e-5)
    for b in batches(3, seed=14):
        step(*b)
    assert m.engine.lagging()
    _ = m.mlp_embedding_collection.embedding_bags["user_id"].weight
    assert not m.engine.lagging()


def test_gradient_accumulation_equals_doubled_loss(monkeypatch):
    """Two backward() calls before one step() accumulate (table rows included): == one
    backward of twice the loss (the same batch; x2 is exact in fp32)."""
    from ncf_amd import optim
    monkeypatch.setattr(optim, "SCHEDULE", "deferred")
    data = batches(6, seed=15)
    crit = torch.nn.BCELoss()
    out = []
    for accumulate in (True, False):
        m = model(seed=23)
        opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-5)
        m.train()
        for u, i, t in data:
            opt.zero_grad()
            if accumulate:
                crit(m(kjt(u, i)), t).backward()
                crit(m(kjt(u, i)), t).backward()
            else:
                (2.0 * crit(m(kjt(u, i)), t)).backward()
            opt.step()
        out.append(snapshot(m, opt))
    for k in out[0][0]:
        torch.testing.assert_close(out[0][0][k], out[1][0][k], rtol=0, atol=1e-7, msg=k)


def test_zero_grad_between_backwards_discards_first(monkeypatch):
    """backward, zero_grad, backward, step == backward, step (the first gradient dropped)."""
    data = batches(4, seed=16)
    crit = torch.nn.BCELoss()
    out = []
    for extra in (True, False):
        m = model(seed=24)
        opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-5)
        m.train()
        for s, (u, i, t) in enumerate(data):
            if extra:
                crit(m(kjt(data[-1 - s][0], data[-1 - s][1])), data[-1 - s][2]).backward()
                opt.zero_grad(set_to_none=(s % 2 == 0))
            loss = crit(m(kjt(u, i)), t)
            opt.zero_grad(set_to_none=(s % 2 == 1))
            loss.backward()
            opt.step()
        out.append(snapshot(m, opt))
    assert_same(out[0], out[1])


def test_out_of_range_id_in_training_raises_without_sync():
    m = model(seed=25)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    crit = torch.nn.BCELoss()
    u, i, t = batches(1, seed=17)[0]
    i = i.clone()
    i[3] = I + 5
    m.train()
    with pytest.raises(IndexError):
        for _ in range(4 * m.engine.ID_CHECK_EVERY):
            loss = crit(m(kjt(u, i)), t)
            opt.zero_grad()
            loss.backward()
            opt.step()
            torch.cuda.synchronize()
    m.validate_ids = "sync"
    with pytest.raises(IndexError):
        m(kjt(u, i))


def test_bad_id_in_a_rare_batch_geometry_is_reported():
    """The id-error flag is engine-wide: a bad id in a short last batch (its own workspace,
    used once) is reported by the asynchronous check of later full batches, or at the latest
    by the next table read (state_dict), and the flag that fired is the one cleared."""
    m = model()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-5)
    crit = torch.nn.BCELoss()
    data = batches(2, seed=31)
    u, i, t = data[0]
    short = (u[:2 * M].clone(), i[:2 * M].clone(), t[:2 * M])
    short[1][1] = I + 7
    m.train()

    def step(u, i, t):
        loss = crit(m(kjt(u, i)), t)
        opt.zero_grad()
        loss.backward()
        opt.step()
    step(*short)
    with pytest.raises(IndexError):
        for _ in range(4 * m.engine.ID_CHECK_EVERY):
            step(*data[1])
            torch.cuda.synchronize()
    step(*data[1])                       # cleared: the following good steps run
    m.state_dict()
    step(*short)                         # one more bad short batch, then a table read
    torch.cuda.synchronize()
    with pytest.raises(IndexError):
        m.state_dict()
    m.state_dict()


def test_fused_step_reports_bad_ids():
    """FusedTrainStep checks ids asynchronously too (it used to never look at the flag)."""
    from ncf_amd.trainer import FusedTrainStep
    m = model()
    step = FusedTrainStep(m, lr=1e-3, weight_decay=1e-5)
    u, i, t = batches(1, seed=32)[0]
    i = i.clone()
    i[7] = I
    with pytest.raises(IndexError):
        for _ in range(4 * m.engine.ID_CHECK_EVERY):
            step(u, i, t)
            torch.cuda.synchronize()


def test_trainer_train_epoch_runs_reference_loop():
    """ModelTrainer.train_epoch (trainer.py:216-337 mirror) over a device-sampled epoch."""
    from ncf_amd.trainer import ModelTrainer
    m = ncf.AdvancedNCF(U, I, 5, 24, 64, 64, 32, [256, 128, 64], 4, 0.2, 4)
    tr = ModelTrainer(m, {"num_users": U, "num_products": I, "batch_size": B,
                          "learning_rate": 1e-3, "weight_decay": 1e-5})
    loader = []
    for u, i, t in batches(8, seed=18):
        loader.append((kjt(u, i), t))
    a = tr.train_epoch(loader)
    b = tr.train_epoch(loader)
    assert np.isfinite(a) and np.isfinite(b) and b < a
    ev = tr.validate([(kjt(u[::M].contiguous(), i[::M].contiguous()), t[::M].contiguous())
                      for (u, i, t) in batches(3, seed=19)])
    assert np.isfinite(ev["val_loss"]) and 0.0 <= ev["accuracy"] <= 1.0


def test_trainer_train_epochs_checkpoints_and_resume(tmp_path):
    """ModelTrainer.train (trainer.py:412-546 mirror): per-epoch history, checkpoint_epoch_{e}.pt
    every epoch and best_model.pt on improvement; a second trainer pointed at the same directory
    resumes from the latest checkpoint (trainer.py:448-451, _load_checkpoint returns epoch + 1),
    runs only the remaining epochs and ends where the uninterrupted run ends; patience 0 stops
    after the first epoch (trainer.py:515)."""
    from ncf_amd.trainer import ModelTrainer
    cfg = {"num_users": U, "num_products": I, "batch_size": B, "learning_rate": 1e-3,
           "weight_decay": 1e-5}
    loader = [(kjt(u, i), t) for u, i, t in batches(4, seed=31)]
    val = [(kjt(u[::M].contiguous(), i[::M].contiguous()), t[::M].contiguous())
           for (u, i, t) in batches(2, seed=32)]

    full = ModelTrainer(model(seed=41), cfg)
    h = full.train(loader, val, num_epochs=3, early_stopping_patience=10,
                   checkpoint_dir=str(tmp_path / "a"))
    assert len(h["train_loss"]) == len(h["val_loss"]) == len(h["learning_rate"]) == 3
    assert all(np.isfinite(x) for x in h["train_loss"] + h["val_loss"])
    assert h["train_loss"][2] < h["train_loss"][0]
    for e in (1, 2, 3):
        assert (tmp_path / "a" / f"checkpoint_epoch_{e}.pt").exists()
    assert (tmp_path / "a" / "best_model.pt").exists()
    ref = {k: v.detach().cpu().clone() for k, v in full.model.state_dict().items()}

    first = ModelTrainer(model(seed=41), cfg)
    first.train(loader, val, num_epochs=2, early_stopping_patience=10,
                checkpoint_dir=str(tmp_path / "b"))
    resumed = ModelTrainer(model(seed=42), cfg)       # other weights: the checkpoint replaces them
    h2 = resumed.train(loader, val, num_epochs=3, early_stopping_patience=10,
                       checkpoint_dir=str(tmp_path / "b"))
    assert len(h2["train_loss"]) == 1
    assert (tmp_path / "b" / "checkpoint_epoch_3.pt").exists()
    got = resumed.model.state_dict()
    for k in ref:
        torch.testing.assert_close(got[k].cpu(), ref[k], rtol=0, atol=1e-6, msg=k)

    stop = ModelTrainer(model(seed=43), cfg)
    h3 = stop.train(loader, val, num_epochs=5, early_stopping_patience=0)
    assert len(h3["train_loss"]) == 1
