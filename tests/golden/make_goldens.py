#!/usr/bin/env python3
"""Generate the golden fixtures F1-F5 from the REFERENCE implementation.

Run only in the survey/build container (it imports /root/reference, which never
travels to the GPU box):

    python tests/golden/make_goldens.py --reference /root/reference

What it does
  * puts the offline torchrec stand-in (tests/golden/_standin) first on sys.path and
    imports the reference's own ``src/model/architecture.py`` (AdvancedNCF,
    MultiHeadAttention, TemporalEncoding);
  * loads the reference's demo checkpoint
    (src/inference/demo/train_20241225_002713_model/, an *unzipped* torch.save archive)
    with ``torch.load(weights_only=True)`` after re-packing the directory into the zip
    container torch expects (a container conversion only; nothing in the file executes);
  * restates ModelTrainer.train_epoch's inner step (src/model/trainer.py:253-285:
    model.train(); out = model(kjt); nn.BCELoss; zero_grad; backward; no clipping
    (the hasattr(dict, ...) guard at :279 is always False); Adam.step) because trainer.py
    itself cannot be imported offline (google.cloud, torchrec.distributed).

Fixtures written to tests/golden/*.npz (inputs and expected outputs only):
  F1 f1_eval_demo.npz      eval forward known-answer: 1000 pairs of the reference's
                           src/inference/demo/data/predictions.csv, the checkpoint rows
                           they touch (ids remapped to 0..n-1), reference re-run outputs
  F2 f2_train_c2.npz       train goldens, C2 architecture at small scale, dropout=0
  F3 f3_train_c1.npz       train goldens, C1 architecture (D=16, H=1, MLP [64,32])
  F4 f4_ops.npz            MultiHeadAttention (L=5 and L=50) and TemporalEncoding fwd+bwd
  F5 f5_scoring.npz        forward_simple(hour=None) 8 users x 366 items + top-10,
                           get_user_embeddings / get_product_embeddings on the demo model
  F6 f6_hour.npz           forward_simple(hour=h) on the demo model (users of F5) x 366 items.
                           The reference draws a fresh nn.Linear(T, D) inside every call
                           (architecture.py:437-442); seeding torch right before the call fixes
                           its init, and the same seed reproduces its weights, stored here.
  F7 f7_metrics.npz        src/utils/metrics.py calculate_metrics on seeded predictions (no ties)
  F8 f8_negatives.npz      src/model/data_prep.py SheetzDataset on a synthetic interaction log:
                           the train interaction list, product_weights, user histories, and the
                           empirical distribution of 40,000 _sample_negative draws (np seed 0)
                           for a few (user, positive) pairs
  F9 f9_batches.npz        src/model/data_prep.py ConsistentBatchSampler: the index batches of
                           several (dataset_size, batch_size) cases, unshuffled and shuffled
                           under np.random.seed (last-batch padding with repeats of the batch)
"""
import argparse
import csv
import io
import os
import sys
import zipfile

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
DEMO = "src/inference/demo/train_20241225_002713_model"
PRED = "src/inference/demo/data/predictions.csv"


def import_reference(ref):
    sys.path.insert(0, os.path.join(HERE, "_standin"))
    sys.path.insert(1, ref)
    from src.model.architecture import AdvancedNCF, MultiHeadAttention, TemporalEncoding
    from torchrec.sparse.jagged_tensor import KeyedJaggedTensor
    return AdvancedNCF, MultiHeadAttention, TemporalEncoding, KeyedJaggedTensor


def load_demo_state(ref):
    src = os.path.join(ref, DEMO)
    buf = io.BytesIO()
    with zipfile.ZipFile(buf, "w", zipfile.ZIP_STORED) as z:
        for root, _, files in os.walk(src):
            for f in sorted(files):
                p = os.path.join(root, f)
                z.write(p, "archive/" + os.path.relpath(p, src))
    buf.seek(0)
    return torch.load(buf, map_location="cpu", weights_only=True)


TABLES = {
    "mf_embedding_collection.embedding_bags.user_id.weight": "user",
    "mlp_embedding_collection.embedding_bags.user_id.weight": "user",
    "mf_embedding_collection.embedding_bags.product_id.weight": "item",
    "mlp_embedding_collection.embedding_bags.product_id.weight": "item",
}


def sd_to_np(sd, prefix=""):
    return {prefix + k: v.detach().cpu().numpy().astype(np.float32) for k, v in sd.items()}


def kjt_for(KJT, users, items):
    n = users.numel()
    return KJT.from_lengths_sync(keys=["user_id", "product_id"],
                                 values=torch.cat([users, items]).long(),
                                 lengths=torch.ones(2 * n, dtype=torch.long))


# ----------------------------------------------------------------------------- F1
def make_f1(ref, AdvancedNCF, KJT, sd):
    rows = list(csv.DictReader(open(os.path.join(ref, PRED))))
    u = np.array([int(r["user_id"]) for r in rows], np.int64)
    i = np.array([int(r["product_id"]) for r in rows], np.int64)
    lab = np.array([int(r["label"]) for r in rows], np.int64)
    csv_pred = np.array([float(r["prediction"]) for r in rows], np.float32)
    uu, ur = np.unique(u, return_inverse=True)
    iu, ir = np.unique(i, return_inverse=True)
    # reference re-run on the full checkpoint, batches of 32 (local_inference.py:121-129)
    model = AdvancedNCF(8031, 366, 5, 24, 64, 64, 32, [256, 128, 64], 4, 0.2, 4)
    model.load_state_dict(sd, strict=True)
    model.eval()
    outs = []
    with torch.no_grad():
        for s in range(0, len(u), 32):
            outs.append(model(kjt_for(KJT, torch.from_numpy(u[s:s + 32]),
                                      torch.from_numpy(i[s:s + 32]))).reshape(-1))
    ref_pred = torch.cat(outs).numpy()
    print(f"F1: max|ref_rerun - predictions.csv| = {np.abs(ref_pred - csv_pred).max():.3e}")
    sub = {}
    for k, v in sd.items():
        if k in TABLES:
            v = v[torch.from_numpy(uu if TABLES[k] == "user" else iu)]
        sub["sd/" + k] = v.numpy().astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "f1_eval_demo.npz"),
                        user_ids=ur.astype(np.int64), item_ids=ir.astype(np.int64),
                        user_ids_orig=u, item_ids_orig=i, label=lab,
                        csv_pred=csv_pred, ref_pred=ref_pred.astype(np.float32),
                        cfg=np.array([len(uu), len(iu), 5, 24, 64, 64, 32, 4], np.int64),
                        hidden=np.array([256, 128, 64], np.int64), **sub)


# ----------------------------------------------------------------------------- F2/F3
ZONE = 1e-6   # = tests/parity.py ZONE


def make_batch(g, U, I, B, M):
    users = torch.randint(0, U, (B,), generator=g)
    pos = torch.randint(0, I, (B,), generator=g)
    neg = torch.randint(0, I, (B, M - 1), generator=g)
    uid = users.repeat_interleave(M)                          # data_prep.py:201
    iid = torch.cat([pos[:, None], neg], 1).reshape(-1)       # data_prep.py:202
    t = torch.zeros(B, M)
    t[:, 0] = 1.0                                             # data_prep.py:214-215
    return uid, iid, t.reshape(-1, 1)


def make_train(fname, AdvancedNCF, KJT, U, I, D, T, hidden, H, B, M, steps, seed, lr, wd):
    torch.manual_seed(seed)
    model = AdvancedNCF(U, I, 5, 24, D, D, T, hidden, H, 0.0, M - 1)
    init = {k: v.clone() for k, v in model.state_dict().items()}
    opt = torch.optim.Adam(model.parameters(), lr=lr, weight_decay=wd)   # trainer.py:71-75
    crit = nn.BCELoss()                                                  # trainer.py:78
    g = torch.Generator().manual_seed(seed + 1)
    out = {}
    names = [n for n, _ in model.named_parameters()]
    for s in range(steps):
        uid, iid, t = make_batch(g, U, I, B, M)
        out[f"step{s}/user_ids"] = uid.numpy()
        out[f"step{s}/item_ids"] = iid.numpy()
        out[f"step{s}/targets"] = t.numpy()
        model.train()
        prob = model(kjt_for(KJT, uid, iid))
        loss = crit(prob, t)
        opt.zero_grad()
        loss.backward()
        out[f"step{s}/prob"] = prob.detach().numpy()
        out[f"step{s}/loss"] = np.float32(loss.item())
        # sign-flip zone of THIS step (tests/parity.py): elements whose effective Adam
        # gradient g + wd * p is below ZONE while g itself is not exactly 0 (summation noise
        # decides its sign), as packed bits per parameter
        for n, p in model.named_parameters():
            if p.grad is not None:
                z = ((p.grad + wd * p.detach()).abs() < ZONE) & (p.grad != 0)
                out[f"zone{s}/{n}"] = np.packbits(z.numpy().reshape(-1))
        if s == 0:
            for n, p in model.named_parameters():
                if p.grad is not None:
                    out["grad0/" + n] = p.grad.numpy().copy()
            out["grad_none0"] = np.array([n for n, p in model.named_parameters()
                                          if p.grad is None])
        opt.step()
        if s in (0, steps - 1):
            tag = f"after{s}"
            for n, p in model.named_parameters():
                st = opt.state.get(p)
                if not st:      # grad None -> Adam skips it; equals init (checked by tests)
                    continue
                out[f"{tag}/param/{n}"] = p.detach().numpy().copy()
                if s == steps - 1:
                    out[f"{tag}/exp_avg/{n}"] = st["exp_avg"].numpy().copy()
                    out[f"{tag}/exp_avg_sq/{n}"] = st["exp_avg_sq"].numpy().copy()
    # eval forward (M = 1) on the final weights
    model.eval()
    with torch.no_grad():
        ge = torch.Generator().manual_seed(seed + 2)
        eu = torch.randint(0, U, (33,), generator=ge)
        ei = torch.randint(0, I, (33,), generator=ge)
        out["eval/user_ids"] = eu.numpy()
        out["eval/item_ids"] = ei.numpy()
        out["eval/prob"] = model(kjt_for(KJT, eu, ei)).numpy()
        out["eval/simple"] = model.forward_simple(eu, ei).numpy()
    for k, v in init.items():
        out["init/" + k] = v.numpy()
    out["param_names"] = np.array(names)
    out["cfg"] = np.array([U, I, D, T, H, B, M, steps], np.int64)
    out["hidden"] = np.array(hidden, np.int64)
    out["hparams"] = np.array([lr, wd], np.float64)
    np.savez_compressed(os.path.join(HERE, fname), **out)
    print(f"{fname}: losses", [float(out[f'step{s}/loss']) for s in range(steps)])


# ----------------------------------------------------------------------------- F4
def make_f4(MultiHeadAttention, TemporalEncoding):
    out = {}
    for tag, (Bn, L, D, H) in {"mha5": (4, 5, 64, 4), "mha50": (4, 50, 64, 4),
                               "mha5_h1": (3, 5, 16, 1)}.items():
        torch.manual_seed(100 + L + H)
        m = MultiHeadAttention(D, H, dropout=0.0)
        q = torch.randn(Bn, L, D, requires_grad=True)
        k = torch.randn(Bn, L, D, requires_grad=True)
        v = torch.randn(Bn, L, D, requires_grad=True)
        y = m(q, k, v)
        gy = torch.randn_like(y)
        y.backward(gy)
        out[f"{tag}/q"], out[f"{tag}/k"], out[f"{tag}/v"] = q.detach().numpy(), k.detach().numpy(), v.detach().numpy()
        out[f"{tag}/y"], out[f"{tag}/gy"] = y.detach().numpy(), gy.numpy()
        out[f"{tag}/gq"], out[f"{tag}/gk"], out[f"{tag}/gv"] = q.grad.numpy(), k.grad.numpy(), v.grad.numpy()
        for n, p in m.named_parameters():
            out[f"{tag}/w/{n}"] = p.detach().numpy()
            out[f"{tag}/gw/{n}"] = p.grad.numpy()
        out[f"{tag}/shape"] = np.array([Bn, L, D, H], np.int64)
    torch.manual_seed(7)
    te = TemporalEncoding(32)
    n = 257
    hour = torch.randint(0, 24, (n,))
    day = torch.randint(0, 7, (n,))
    month = torch.randint(0, 12, (n,))
    days = torch.randint(0, 2000, (n,))                  # >= 365 exercises the modulo
    days[:4] = torch.tensor([0, 364, 365, 730])
    y = te(hour, day, month, days)
    gy = torch.randn_like(y)
    y.backward(gy)
    out.update({"te/hour": hour.numpy(), "te/day": day.numpy(), "te/month": month.numpy(),
                "te/days_since": days.numpy(), "te/y": y.detach().numpy(), "te/gy": gy.numpy()})
    for nme, p in te.named_parameters():
        out["te/w/" + nme] = p.detach().numpy()
        out["te/gw/" + nme] = p.grad.numpy()
    out["te/pe"] = te.pe.numpy()
    np.savez_compressed(os.path.join(HERE, "f4_ops.npz"), **out)
    print("F4 written")


# ----------------------------------------------------------------------------- F5
def make_f5(AdvancedNCF, KJT, sd):
    model = AdvancedNCF(8031, 366, 5, 24, 64, 64, 32, [256, 128, 64], 4, 0.2, 4)
    model.load_state_dict(sd, strict=True)
    model.eval()
    users = torch.tensor([5021, 0, 17, 4096, 8030, 1234, 777, 3141])
    items = torch.arange(366)
    with torch.no_grad():
        scores = torch.stack([model.forward_simple(torch.full((366,), int(u)), items)
                              for u in users])
        top_s, top_i = scores.topk(10, dim=1)
        ue = model.get_user_embeddings({"user_features": kjt_for(KJT, users, torch.zeros_like(users))})
        pid = torch.tensor([0, 5, 179, 365])
        dept = torch.tensor([0, 1, 4, 2])
        cat = torch.tensor([0, 23, 7, 11])
        pe = model.get_product_embeddings({
            "product_features": kjt_for(KJT, torch.zeros_like(pid), pid),
            "category_features": {"department_ids": dept, "category_ids": cat}})
    sub = {}
    for k, v in sd.items():
        if k in TABLES and TABLES[k] == "user":
            v = v[users]
        sub["sd/" + k] = v.numpy().astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "f5_scoring.npz"),
                        users_orig=users.numpy(), scores=scores.numpy(),
                        top_scores=top_s.numpy(), top_items=top_i.numpy(),
                        emb_user_mf=ue["mf"].numpy(), emb_user_mlp=ue["mlp"].numpy(),
                        emb_pids=pid.numpy(), emb_dept=dept.numpy(), emb_cat=cat.numpy(),
                        emb_item_mf=pe["mf"].numpy(), emb_item_mlp=pe["mlp"].numpy(),
                        emb_item_category=pe["category"].numpy(), **sub)
    print("F5 written; top-1 items", top_i[:, 0].tolist())


def make_f6(AdvancedNCF, sd):
    model = AdvancedNCF(8031, 366, 5, 24, 64, 64, 32, [256, 128, 64], 4, 0.2, 4)
    model.load_state_dict(sd, strict=True)
    model.eval()
    f5_users = [5021, 0, 17, 4096, 8030, 1234, 777, 3141]
    calls = [(0, 0), (1, 13), (2, 23), (4, 7)]       # (index into F5's users, hour)
    items = torch.arange(366)
    scores, ws, bs = [], [], []
    with torch.no_grad():
        for c, (ui, hour) in enumerate(calls):
            torch.manual_seed(1000 + c)
            scores.append(model.forward_simple(torch.full((366,), f5_users[ui]), items,
                                               torch.full((366,), hour)))
            torch.manual_seed(1000 + c)
            lin = nn.Linear(32, 64)                   # the projection the call above drew
            ws.append(lin.weight.detach().clone())
            bs.append(lin.bias.detach().clone())
    np.savez_compressed(os.path.join(HERE, "f6_hour.npz"),
                        user_pos=np.array([c[0] for c in calls]), hours=np.array([c[1] for c in calls]),
                        scores=torch.stack(scores).numpy(), proj_w=torch.stack(ws).numpy(),
                        proj_b=torch.stack(bs).numpy())
    print("F6 written; scores[0][:4]", scores[0][:4].tolist())


def make_f7(ref):
    from src.utils.metrics import calculate_metrics
    out = {}
    for name, (B, M, seed) in {"a": (64, 5, 0), "b": (33, 8, 1)}.items():
        g = torch.Generator().manual_seed(seed)
        p = torch.rand(B * M, 1, generator=g)
        t = torch.zeros(B, M)
        t[:, 0] = 1
        t[torch.rand(B, M, generator=g) < 0.15] = 1
        t = t.reshape(-1, 1)
        m = calculate_metrics(p, t, k_values=[1, 5, 10], batch_size=B, negative_samples=M - 1)
        out[f"{name}_pred"] = p.numpy()
        out[f"{name}_targ"] = t.numpy()
        out[f"{name}_shape"] = np.array([B, M])
        out[f"{name}_keys"] = np.array(list(m.keys()))
        out[f"{name}_vals"] = np.array([float(v) for v in m.values()])
    np.savez_compressed(os.path.join(HERE, "f7_metrics.npz"), **out)
    print("F7 written;", dict(zip(out["a_keys"][:4], out["a_vals"][:4])))


def make_f8(ref):
    import pandas as pd
    from src.model.data_prep import SheetzDataset
    rng = np.random.default_rng(8)
    U, I, P = 30, 40, 400
    users = rng.integers(0, U, P)
    prods = np.minimum(rng.zipf(1.4, P) - 1, I - 1)
    days = rng.integers(0, 60, P)
    ts = pd.Timestamp("2024-01-01") + pd.to_timedelta(days, unit="D")
    inter = pd.DataFrame({"user_id": [f"U{u}" for u in users], "product_id": [f"P{p}" for p in prods],
                          "amount": rng.random(P), "transaction_timestamp": ts})
    ufeat = pd.DataFrame({"cardnumber": [f"U{u}" for u in range(U)],
                          "recent_interactions": [0] * U, "preferred_categories": [""] * U})
    pfeat = pd.DataFrame({"product_id": [f"P{p}" for p in range(I)], "total_purchases": [0] * I,
                          "total_revenue": [0.0] * I})
    ds = SheetzDataset(inter, ufeat, pfeat, mode="train", validation_days=10, negative_samples=4)
    il = np.array([(u, p) for u, p, _ in ds.interaction_list], dtype=np.int64)
    hist_u, hist_i = [], []
    for u, items in sorted(ds.user_product_history.items()):
        for i in sorted(items):
            hist_u.append(u)
            hist_i.append(i)
    # a light user, a heavy user (the fallback path), the most popular product as positive
    by_len = sorted(ds.user_product_history, key=lambda u: len(ds.user_product_history[u]))
    picks = [by_len[0], by_len[len(by_len) // 2], by_len[-1]]
    pairs, counts = [], []
    np.random.seed(0)
    for u in picks:
        pos = sorted(ds.user_product_history[u])[0]
        c = np.zeros(ds.num_products, dtype=np.int64)
        for _ in range(40_000):
            c[ds._sample_negative(u, pos)] += 1
        pairs.append((u, pos))
        counts.append(c)
    np.savez_compressed(os.path.join(HERE, "f8_negatives.npz"), interactions=il,
                        num_users=ds.num_users, num_products=ds.num_products,
                        product_weights=ds.product_weights, hist_u=np.array(hist_u),
                        hist_i=np.array(hist_i), pairs=np.array(pairs), counts=np.array(counts))
    print("F8 written;", len(il), "train interactions; pairs", pairs)


def make_f9(ref):
    from src.model.data_prep import ConsistentBatchSampler
    cases = [(10, 4, 0), (10, 8, 0), (8, 4, 0), (1, 4, 0), (37, 5, 0), (10, 3, 1), (23, 7, 1),
             (6, 20, 1)]
    flat, bounds, meta = [], [0], []
    for size, bs, shuffle in cases:
        if shuffle:
            np.random.seed(size * 100 + bs)
        sm = ConsistentBatchSampler(size, bs, shuffle=bool(shuffle))
        batches = list(iter(sm))
        assert len(batches) == len(sm)
        for b in batches:
            flat.extend(int(x) for x in b)
            bounds.append(len(flat))
        meta.append((size, bs, shuffle, len(batches)))
    np.savez_compressed(os.path.join(HERE, "f9_batches.npz"), cases=np.array(meta, dtype=np.int64),
                        indices=np.array(flat, dtype=np.int64), bounds=np.array(bounds, dtype=np.int64))
    print("F9 written;", len(meta), "cases")


def make_train_fixtures(AdvancedNCF, KJT):
    make_train("f2_train_c2.npz", AdvancedNCF, KJT, U=300, I=120, D=64, T=32,
               hidden=[256, 128, 64], H=4, B=8, M=5, steps=3, seed=0, lr=1e-3, wd=1e-5)
    make_train("f3_train_c1.npz", AdvancedNCF, KJT, U=200, I=300, D=16, T=32,
               hidden=[64, 32], H=1, B=16, M=5, steps=3, seed=1, lr=1e-3, wd=1e-5)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--only", default=None, help="write one fixture only (e.g. f6)")
    a = ap.parse_args()
    torch.set_num_threads(8)
    AdvancedNCF, MHA, TE, KJT = import_reference(a.reference)
    sd = load_demo_state(a.reference)
    if a.only == "f6":
        make_f6(AdvancedNCF, sd)
        return
    if a.only == "train":
        make_train_fixtures(AdvancedNCF, KJT)
        return
    if a.only in ("f7", "f8", "f9"):
        {"f7": make_f7, "f8": make_f8, "f9": make_f9}[a.only](a.reference)
        return
    make_f1(a.reference, AdvancedNCF, KJT, sd)
    make_train_fixtures(AdvancedNCF, KJT)
    make_f4(MHA, TE)
    make_f5(AdvancedNCF, KJT, sd)
    make_f6(AdvancedNCF, sd)
    make_f7(a.reference)
    make_f8(a.reference)
    make_f9(a.reference)


if __name__ == "__main__":
    main()
