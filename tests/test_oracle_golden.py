"""The CPU oracle (oracle/ncf_oracle.py) pinned against the reference's golden vectors F1-F5
(tests/golden/make_goldens.py ran the reference itself).  CPU only."""
import numpy as np
import pytest
import torch

from oracle import ncf_oracle as O
from tests.conftest import sub
from tests.parity import assert_moment_close, assert_params_close, zone_masks


def T(d):
    return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in d.items()}


def test_f1_eval_known_answer(f1):
    p = T(sub(f1, "sd/"))
    u = torch.from_numpy(f1["user_ids"])
    i = torch.from_numpy(f1["item_ids"])
    prob = O.forward(p, u, i, training=False, negative_samples=4, num_heads=4,
                     temporal_dim=32, n_layers=3).reshape(-1).numpy()
    # the reference's committed predictions.csv (produced by local_inference.py:121-136)
    assert np.abs(prob - f1["csv_pred"]).max() < 1e-6
    assert np.abs(prob - f1["ref_pred"]).max() < 1e-6


def test_f1_factorised_scoring(f1):
    p = T(sub(f1, "sd/"))
    u = torch.from_numpy(f1["user_ids"])
    i = torch.from_numpy(f1["item_ids"])
    full = O.score_factorised(p, torch.arange(p[O.K_MF_U].shape[0]),
                              torch.arange(p[O.K_MF_I].shape[0]), temporal_dim=32, n_layers=3)
    assert np.abs(full[u, i].numpy() - f1["csv_pred"]).max() < 1e-6


@pytest.mark.parametrize("fx,heads,nl", [("f2", 4, 3), ("f3", 1, 2)])
def test_train_goldens(fx, heads, nl, request):
    g = request.getfixturevalue(fx)
    U, I, D, Tt, H, B, M, steps = [int(x) for x in g["cfg"]]
    lr, wd = [float(x) for x in g["hparams"]]
    p = T(sub(g, "init/"))
    init = {k: v.clone() for k, v in p.items()}
    opt = O.AdamState(lr=lr, weight_decay=wd)
    for s in range(steps):
        u = torch.from_numpy(g[f"step{s}/user_ids"])
        i = torch.from_numpy(g[f"step{s}/item_ids"])
        t = torch.from_numpy(g[f"step{s}/targets"])
        prob, loss, grads = O.train_step(p, opt, u, i, t, negative_samples=M - 1, num_heads=H,
                                         temporal_dim=Tt, n_layers=nl)
        assert np.abs(prob.numpy() - g[f"step{s}/prob"]).max() < 1e-6
        assert abs(float(loss) - float(g[f"step{s}/loss"])) < 1e-6
        if s == 0:
            gold = sub(g, "grad0/")
            assert set(gold) == set(grads)
            for k, v in gold.items():
                np.testing.assert_allclose(grads[k].numpy(), v, rtol=1e-4, atol=1e-7, err_msg=k)
            assert set(g["grad_none0"].tolist()) == set(p) - set(gold) - {"temporal_encoding.pe"}
        if s in (0, steps - 1):
            for k, v in sub(g, f"after{s}/param/").items():
                assert_params_close(k, p[k].numpy(), v, zone_masks(g, k, s + 1), lr)
    for k, v in sub(g, f"after{steps - 1}/exp_avg/").items():
        assert_moment_close(k, opt.state[k]["exp_avg"].numpy(), v, zone_masks(g, k, steps))
    for k, v in sub(g, f"after{steps - 1}/exp_avg_sq/").items():
        assert_moment_close(k, opt.state[k]["exp_avg_sq"].numpy(), v, zone_masks(g, k, steps),
                            atol=1e-12)
    for k in g["grad_none0"].tolist():        # grad None -> untouched by Adam
        assert torch.equal(p[k], init[k])
    e_u, e_i = torch.from_numpy(g["eval/user_ids"]), torch.from_numpy(g["eval/item_ids"])
    ev = O.forward(p, e_u, e_i, training=False, negative_samples=M - 1, num_heads=H,
                   temporal_dim=Tt, n_layers=nl)
    assert np.abs(ev.numpy() - g["eval/prob"]).max() < 2e-6
    assert np.abs(g["eval/simple"] - g["eval/prob"][:, 0]).max() < 1e-6


@pytest.mark.parametrize("tag", ["mha5", "mha50", "mha5_h1"])
def test_f4_mha(f4, tag):
    Bn, L, D, H = [int(x) for x in f4[f"{tag}/shape"]]
    w = {k: torch.from_numpy(v).requires_grad_(True) for k, v in sub(f4, f"{tag}/w/").items()}
    q, k, v = [torch.from_numpy(f4[f"{tag}/{n}"]).requires_grad_(True) for n in "qkv"]
    y = O.mha(w, "", q, k, v, H)
    np.testing.assert_allclose(y.detach().numpy(), f4[f"{tag}/y"], atol=1e-5, rtol=1e-5)
    y.backward(torch.from_numpy(f4[f"{tag}/gy"]))
    for n, t in zip("qkv", (q, k, v)):
        np.testing.assert_allclose(t.grad.numpy(), f4[f"{tag}/g{n}"], atol=1e-5, rtol=1e-4)
    for n, t in w.items():
        np.testing.assert_allclose(t.grad.numpy(), f4[f"{tag}/gw/{n}"], atol=1e-5, rtol=1e-4)


def test_f4_temporal(f4):
    w = {"temporal_encoding." + k: torch.from_numpy(v).requires_grad_(True)
         for k, v in sub(f4, "te/w/").items()}
    pe = O.sinusoid_pe(365, 32)
    assert np.abs(pe.numpy() - f4["te/pe"]).max() == 0.0
    w["temporal_encoding.pe"] = pe
    args = [torch.from_numpy(f4[f"te/{n}"]) for n in ("hour", "day", "month", "days_since")]
    y = O.temporal_encoding(w, *args)
    np.testing.assert_allclose(y.detach().numpy(), f4["te/y"], atol=1e-6)
    y.backward(torch.from_numpy(f4["te/gy"]))
    for n in ("hour_embed.weight", "day_embed.weight", "month_embed.weight"):
        np.testing.assert_allclose(w["temporal_encoding." + n].grad.numpy(), f4["te/gw/" + n],
                                   atol=1e-5, rtol=1e-5)


def test_f5_scoring(f5):
    p = T(sub(f5, "sd/"))
    nu = p[O.K_MF_U].shape[0]
    items = torch.arange(p[O.K_MF_I].shape[0])
    s = O.score_factorised(p, torch.arange(nu), items, temporal_dim=32, n_layers=3)
    np.testing.assert_allclose(s.numpy(), f5["scores"], atol=1e-6)
    lit = torch.stack([O.forward_simple(p, torch.full_like(items, u), items, num_heads=4,
                                        temporal_dim=32, n_layers=3) for u in range(nu)])
    np.testing.assert_allclose(lit.numpy(), f5["scores"], atol=1e-6)
    ts, ti = lit.topk(10, dim=1)
    assert (ti.numpy() == f5["top_items"]).all()


def test_f6_forward_simple_hour(f5, f6):
    """forward_simple(hour=h): the reference's per-call random projection, reproduced by seed and
    stored in F6, pins the restatement of the hour path (architecture.py:432-468)."""
    p = T(sub(f5, "sd/"))
    items = torch.arange(p[O.K_MF_I].shape[0])
    for c in range(len(f6["hours"])):
        u = torch.full_like(items, int(f6["user_pos"][c]))
        h = torch.full_like(items, int(f6["hours"][c]))
        s = O.forward_simple_hour(p, u, items, h, torch.from_numpy(f6["proj_w"][c]),
                                  torch.from_numpy(f6["proj_b"][c]), num_heads=4, n_layers=3)
        np.testing.assert_allclose(s.numpy(), f6["scores"][c], atol=1e-6)


def test_f7_metrics_oracle(f7):
    """oracle.ranking_metrics == the reference's calculate_metrics (F7) on the same inputs."""
    for c in ("a", "b"):
        B, M = f7[f"{c}_shape"].tolist()
        p = f7[f"{c}_pred"].reshape(B, M).tolist()
        t = f7[f"{c}_targ"].reshape(B, M).tolist()
        got = O.ranking_metrics(p, t, [1, 5, 10])
        keys = [str(k) for k in f7[f"{c}_keys"]]
        assert list(got) == keys
        np.testing.assert_allclose([got[k] for k in keys], f7[f"{c}_vals"], atol=1e-6)


def test_f8_negative_sampling_oracle(f8):
    """oracle weights == SheetzDataset.product_weights; oracle.negative_distribution matches
    40,000 of the reference's own _sample_negative draws per pair (6 sigma)."""
    inter = f8["interactions"]
    I = int(f8["num_products"])
    w = O.inverse_popularity_weights(inter[:, 1].tolist(), I)
    np.testing.assert_allclose(w, f8["product_weights"], rtol=1e-12)
    hu, hi = f8["hist_u"], f8["hist_i"]
    for (u, pos), cnt in zip(f8["pairs"], f8["counts"]):
        exp = O.negative_distribution(w, hi[hu == u].tolist(), int(pos))
        n = cnt.sum()
        emp = cnt / n
        sig = np.sqrt(np.maximum(exp * (1 - exp), 1e-12) / n)
        assert np.all(np.abs(emp - exp) <= 6 * sig + 1e-9)
