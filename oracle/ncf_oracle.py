"""CPU oracle for the AdvancedNCF hot path — TEST INFRASTRUCTURE ONLY.

This module is a from-scratch fp32 restatement, in plain PyTorch-on-CPU functional ops, of
the reference's AdvancedNCF training/scoring math.  It is the *checker*: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it, and never
as the thing measured or shipped.  The product path (the ``ncf_amd`` package) never imports it
and fails loudly when its HIP library is missing.

Parity pin: ``tests/test_oracle_golden.py`` checks every function here against the golden
fixtures F1-F6 that ``tests/golden/make_goldens.py`` produced by running the reference itself
(including the reference's own committed known answer ``src/inference/demo/data/predictions.csv``).

Citations are into the reference (ethanshenley/Neural-Collaborative-Filtering-Demo).
Parameters travel as a flat dict keyed by the reference's 62 state_dict names.
"""
import math
from typing import Dict, Optional

import torch
import torch.nn.functional as F

Tensor = torch.Tensor

K_MF_U = "mf_embedding_collection.embedding_bags.user_id.weight"
K_MF_I = "mf_embedding_collection.embedding_bags.product_id.weight"
K_MLP_U = "mlp_embedding_collection.embedding_bags.user_id.weight"
K_MLP_I = "mlp_embedding_collection.embedding_bags.product_id.weight"
ATT = "user_product_attention."
LN_EPS = 1e-5


def layer_norm(x: Tensor, g: Tensor, b: Tensor) -> Tensor:
    """nn.LayerNorm(D), eps 1e-5 (architecture.py:144-145, 255-256; MLP LNs :237)."""
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + LN_EPS) * g + b


def linear(x: Tensor, w: Tensor, b: Tensor) -> Tensor:
    return x @ w.t() + b


def mha(p: Dict[str, Tensor], pre: str, q_in: Tensor, k_in: Tensor, v_in: Tensor,
        num_heads: int, drop_mask: Optional[Tensor] = None,
        mask: Optional[Tensor] = None) -> Tensor:
    """MultiHeadAttention.forward (architecture.py:35-57): per-head softmax(QK^T/sqrt(hd))V,
    dropout on the weights (:51), merge heads, out_proj.  q_in/k_in/v_in: [B, L, D].  ``mask``
    (:36, :47-48): scores.masked_fill(mask == 0, -inf), broadcast against [B, H, L, L]."""
    B, L, D = q_in.shape
    hd = D // num_heads
    q = linear(q_in, p[pre + "q_proj.weight"], p[pre + "q_proj.bias"]).view(B, -1, num_heads, hd).transpose(1, 2)
    k = linear(k_in, p[pre + "k_proj.weight"], p[pre + "k_proj.bias"]).view(B, -1, num_heads, hd).transpose(1, 2)
    v = linear(v_in, p[pre + "v_proj.weight"], p[pre + "v_proj.bias"]).view(B, -1, num_heads, hd).transpose(1, 2)
    s = (q @ k.transpose(-2, -1)) / math.sqrt(hd)               # :33, :45
    if mask is not None:
        s = s.masked_fill(mask == 0, float("-inf"))              # :47-48
    a = torch.softmax(s, dim=-1)                                 # :50
    if drop_mask is not None:
        a = a * drop_mask
    o = (a @ v).transpose(1, 2).contiguous().view(B, -1, D)      # :54-55
    return linear(o, p[pre + "out_proj.weight"], p[pre + "out_proj.bias"])


def temporal_encoding(p: Dict[str, Tensor], hour, day, month, days_since, pre="temporal_encoding.") -> Tensor:
    """TemporalEncoding.forward (architecture.py:86-94) incl. the sinusoidal pe buffer (:79-84)."""
    t = p[pre + "hour_embed.weight"][hour] + p[pre + "day_embed.weight"][day] + p[pre + "month_embed.weight"][month]
    return t + p[pre + "pe"][days_since.long() % p[pre + "pe"].shape[0]]


def sinusoid_pe(max_period: int, dim: int) -> Tensor:
    """architecture.py:79-84."""
    position = torch.arange(max_period).unsqueeze(1)
    div_term = torch.exp(torch.arange(0, dim, 2) * (-math.log(10000.0) / dim))
    pe = torch.zeros(max_period, dim)
    pe[:, 0::2] = torch.sin(position * div_term)
    pe[:, 1::2] = torch.cos(position * div_term)
    return pe


def mlp_tower(p: Dict[str, Tensor], x: Tensor, n_layers: int, masks=None) -> Tensor:
    """self.mlp (architecture.py:230-242): n x [Linear, ReLU, LayerNorm, Dropout]."""
    for l in range(n_layers):
        x = torch.relu(linear(x, p[f"mlp.{4 * l}.weight"], p[f"mlp.{4 * l}.bias"]))
        x = layer_norm(x, p[f"mlp.{4 * l + 2}.weight"], p[f"mlp.{4 * l + 2}.bias"])
        if masks is not None:
            x = x * masks[l]
    return x


def forward(p: Dict[str, Tensor], user_ids: Tensor, item_ids: Tensor, *, training: bool,
            negative_samples: int, num_heads: int, temporal_dim: int, n_layers: int,
            dropout_masks=None) -> Tensor:
    """AdvancedNCF.forward (architecture.py:258-381) on a KJT whose values are
    [user_ids ‖ item_ids] with unit lengths.  Returns probabilities [N, 1]."""
    n = user_ids.numel()
    M = 1 + negative_samples if training else 1                  # :275
    B = n // M                                                   # :276
    u_mf = p[K_MF_U][user_ids]                                   # EBC SUM of one id == row
    i_mf = p[K_MF_I][item_ids]
    u_mlp = p[K_MLP_U][user_ids]
    i_mlp = p[K_MLP_I][item_ids]
    g, b = p["mf_norm.weight"], p["mf_norm.bias"]
    mf_vec = layer_norm(u_mf, g, b) * layer_norm(i_mf, g, b)     # :305-307
    mf_pred = linear(mf_vec, p["mf_output.weight"], p["mf_output.bias"])   # :308
    g, b = p["mlp_norm.weight"], p["mlp_norm.bias"]
    xu = layer_norm(u_mlp, g, b).view(B, M, -1)                  # :311-316
    xi = layer_norm(i_mlp, g, b).view(B, M, -1)
    am = None if dropout_masks is None else dropout_masks.get("attn")
    att = mha(p, ATT, xu, xi, xi, num_heads, am).reshape(n, -1)  # :319-326
    comb = torch.cat([att, torch.zeros(n, temporal_dim)], 1)     # :329-340
    mm = None if dropout_masks is None else dropout_masks.get("mlp")
    h = mlp_tower(p, comb, n_layers, mm)                         # :344
    mlp_pred = linear(h, p["mlp_output.weight"], p["mlp_output.bias"])     # :345
    z = linear(torch.cat([mf_pred, mlp_pred], 1), p["final.0.weight"], p["final.0.bias"])
    return torch.sigmoid(z)                                      # :353-354


def forward_simple(p, user_ids, product_ids, *, num_heads, temporal_dim, n_layers) -> Tensor:
    """AdvancedNCF.forward_simple(hour=None) (architecture.py:409-485) == eval forward."""
    return forward(p, user_ids, product_ids, training=False, negative_samples=0,
                   num_heads=num_heads, temporal_dim=temporal_dim, n_layers=n_layers).squeeze(-1)


def forward_simple_hour(p, user_ids, product_ids, hour, proj_w, proj_b, *, num_heads,
                        n_layers, attn_drop=None, mlp_masks=None) -> Tensor:
    """AdvancedNCF.forward_simple(hour=h) (architecture.py:409-485).  The reference builds a
    fresh nn.Linear(T, D) inside the call when T != D (:437-442); its weights are inputs here.
    Item rows of both paths are scaled by (1 + 0.3 * proj(hour_E[h])) (:444, :456-458); the MLP
    input is [attention ‖ hour_E[h]] (:467-468).  Training mode: ``attn_drop`` = the keep-scales of
    the attention weights ([B, H, 1, 1], :51) and ``mlp_masks`` those of the tower's dropouts."""
    te = p["temporal_encoding.hour_embed.weight"][hour]
    D = p[K_MF_U].shape[1]
    tp = linear(te, proj_w, proj_b) if te.shape[1] != D else te
    g, b = p["mf_norm.weight"], p["mf_norm.bias"]
    u_mf = layer_norm(p[K_MF_U][user_ids], g, b)
    i_mf = layer_norm(p[K_MF_I][product_ids], g, b) * (1 + 0.3 * tp)
    mf_pred = linear(u_mf * i_mf, p["mf_output.weight"], p["mf_output.bias"])
    g, b = p["mlp_norm.weight"], p["mlp_norm.bias"]
    u_mlp = layer_norm(p[K_MLP_U][user_ids], g, b)
    i_mlp = layer_norm(p[K_MLP_I][product_ids], g, b) * (1 + 0.3 * tp)
    att = mha(p, ATT, u_mlp[:, None], i_mlp[:, None], i_mlp[:, None], num_heads,
              drop_mask=attn_drop)[:, 0]
    h = mlp_tower(p, torch.cat([att, te], 1), n_layers, masks=mlp_masks)
    mlp_pred = linear(h, p["mlp_output.weight"], p["mlp_output.bias"])
    z = linear(torch.cat([mf_pred, mlp_pred], 1), p["final.0.weight"], p["final.0.bias"])
    return torch.sigmoid(z).squeeze(-1)


def score_factorised(p, user_ids, item_ids, *, temporal_dim, n_layers):
    """Eval scoring factorised form: with M=1 softmax == 1, so the MLP path
    depends on the item only; the score of (u, i) is
    sigmoid(w0*(LNmf(U_u)*w_mf . LNmf(I_i) + b_mf) + w1*mlp_item(I_i) + b_f).
    Returns [len(user_ids), len(item_ids)]."""
    g, b = p["mf_norm.weight"], p["mf_norm.bias"]
    U = layer_norm(p[K_MF_U][user_ids], g, b) * p["mf_output.weight"][0]
    I = layer_norm(p[K_MF_I][item_ids], g, b)
    mf = U @ I.t() + p["mf_output.bias"][0]
    g, b = p["mlp_norm.weight"], p["mlp_norm.bias"]
    xi = layer_norm(p[K_MLP_I][item_ids], g, b)
    v = linear(xi, p[ATT + "v_proj.weight"], p[ATT + "v_proj.bias"])
    att = linear(v, p[ATT + "out_proj.weight"], p[ATT + "out_proj.bias"])
    h = mlp_tower(p, torch.cat([att, torch.zeros(xi.shape[0], temporal_dim)], 1), n_layers)
    mlp_item = linear(h, p["mlp_output.weight"], p["mlp_output.bias"])[:, 0]
    w = p["final.0.weight"][0]
    return torch.sigmoid(w[0] * mf + w[1] * mlp_item[None, :] + p["final.0.bias"][0])


def bce_loss(prob: Tensor, target: Tensor) -> Tensor:
    """nn.BCELoss() mean reduction, log clamped at -100 (trainer.py:78, :271)."""
    lp = torch.clamp(torch.log(prob), min=-100.0)
    lq = torch.clamp(torch.log(1 - prob), min=-100.0)
    return -(target * lp + (1 - target) * lq).mean()


class AdamState:
    """torch.optim.Adam(model.parameters(), lr, weight_decay) (trainer.py:71-75), single-tensor
    CPU semantics: coupled L2 (g += wd*p), lerp first moment, fp32 scalars from double math,
    and parameters whose grad is None are skipped entirely (the 27 tensors unused by forward)."""

    def __init__(self, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.state: Dict[str, Dict[str, Tensor]] = {}

    def step(self, params: Dict[str, Tensor], grads: Dict[str, Optional[Tensor]]):
        b1, b2 = self.betas
        for k, g in grads.items():
            if g is None:
                continue
            p = params[k]
            st = self.state.setdefault(k, {"step": 0, "exp_avg": torch.zeros_like(p),
                                           "exp_avg_sq": torch.zeros_like(p)})
            st["step"] += 1
            t = st["step"]
            if self.wd != 0:
                g = g.add(p, alpha=self.wd)
            st["exp_avg"].lerp_(g, 1 - b1)
            st["exp_avg_sq"].mul_(b2).addcmul_(g, g, value=1 - b2)
            step_size = self.lr / (1 - b1 ** t)
            denom = (st["exp_avg_sq"].sqrt() / ((1 - b2 ** t) ** 0.5)).add_(self.eps)
            p.addcdiv_(st["exp_avg"], denom, value=-step_size)


def used_param_names(names, n_layers):
    """Parameters that receive a gradient from AdvancedNCF.forward (everything else has
    grad None: category_hierarchy, temporal_encoding, sequence_attention,
    feature_combination — SURVEY fact 4)."""
    unused = ("category_hierarchy.", "temporal_encoding.", "sequence_attention.", "feature_combination.")
    return [n for n in names if not n.startswith(unused)]


def train_step(p: Dict[str, Tensor], opt: AdamState, user_ids, item_ids, targets, *,
               negative_samples, num_heads, temporal_dim, n_layers, dropout_masks=None):
    """One ModelTrainer.train_epoch batch (trainer.py:253-285): forward, BCE, zero_grad,
    backward (autograd on the CPU restatement), no clipping, Adam.step.
    ``p`` holds leaf tensors and is updated in place.  Returns (prob, loss, grads)."""
    names = used_param_names(list(p.keys()), n_layers)
    leaves = {k: (v.detach().requires_grad_(True) if k in names else v) for k, v in p.items()}
    prob = forward(leaves, user_ids, item_ids, training=True, negative_samples=negative_samples,
                   num_heads=num_heads, temporal_dim=temporal_dim, n_layers=n_layers,
                   dropout_masks=dropout_masks)
    loss = bce_loss(prob, targets)
    gl = torch.autograd.grad(loss, [leaves[k] for k in names])
    grads = dict(zip(names, gl))
    with torch.no_grad():
        opt.step(p, grads)
    return prob.detach(), loss.detach(), grads


# ----------------------------------------------------------------------------- 8f: negatives
def inverse_popularity_weights(products, num_products: int):
    """src/model/data_prep.py:95-102 — per-product interaction counts, clamped to >= 1,
    inverted and normalised (float64 numpy, as the reference's np arrays)."""
    import numpy as np
    counts = np.zeros(num_products)
    for p in [int(x) for x in products]:
        counts[p] += 1
    counts = np.maximum(counts, 1)
    w = 1 / counts
    return w / w.sum()


def negative_distribution(weights, history, positive: int, max_attempts: int = 10):
    """Exact distribution of one ``SheetzDataset._sample_negative(user, positive)`` draw
    (data_prep.py:134-161): up to ``max_attempts`` draws from ``weights``, rejecting the positive
    and the user's history; then uniform over the products outside history + {positive}, or —
    when that set is empty — uniform over every product but the positive."""
    import numpy as np
    n = len(weights)
    excluded = set(int(h) for h in history) | {int(positive)}
    ok = np.ones(n, dtype=bool)
    ok[list(excluded)] = False
    r = float(np.sum(np.asarray(weights)[~ok]))        # rejection probability per attempt
    direct = np.where(ok, weights, 0.0) * sum(r ** a for a in range(max_attempts))
    tail = r ** max_attempts
    valid = np.flatnonzero(ok)
    fb = np.zeros(n)
    if valid.size:
        fb[valid] = 1.0 / valid.size
    else:
        fb[:] = 1.0 / (n - 1)
        fb[int(positive)] = 0.0
    return direct + tail * fb


# ----------------------------------------------------------------------------- 8f: metrics
def ranking_metrics(preds, targs, k_values, threshold=0.5):
    """src/utils/metrics.py:9-266 restated per row with plain Python loops (the reference's own
    loop structure), rank order (prediction desc, column asc); AUC as the Mann-Whitney statistic
    with ties counted one half (what sklearn's roc_auc_score computes).  preds / targs: [B][M]
    nested lists of floats."""
    import math
    B, M = len(preds), len(preds[0])
    out = {}
    for k0 in k_values:
        k = min(k0, M)
        hit = nd = mrr = mp = 0.0
        for p, t in zip(preds, targs):
            order = sorted(range(M), key=lambda j: (-p[j], j))[:k]
            rel = [t[j] for j in order]
            hit += 1.0 if any(r == 1 for r in rel) else 0.0
            dcg = sum(r / math.log2(i + 2) for i, r in enumerate(rel))
            ideal = sorted(t, reverse=True)[:k]
            idcg = sum(r / math.log2(i + 2) for i, r in enumerate(ideal))
            nd += 0.0 if idcg <= 0 else dcg / idcg
            first = next((i for i, r in enumerate(rel) if r == 1), None)
            mrr += 0.0 if first is None else 1.0 / (first + 1)
            cum, s, c = 0, 0.0, 0
            for i, r in enumerate(rel):
                if r == 1:
                    cum += 1
                    s += cum / (i + 1)
                    c += 1
            mp += s / max(c, 1) if c else 0.0
        out[f"hit_rate@{k0}"] = hit / B
        out[f"ndcg@{k0}"] = nd / B
        out[f"mrr@{k0}"] = mrr / B
        out[f"map@{k0}"] = mp / B
    flat_p = [x for row in preds for x in row]
    flat_t = [x for row in targs for x in row]
    pos = [x for x, y in zip(flat_p, flat_t) if y == 1]
    neg = [x for x, y in zip(flat_p, flat_t) if y == 0]
    u = sum((1.0 if a > b else 0.5 if a == b else 0.0) for a in pos for b in neg)
    out["auc"] = u / (len(pos) * len(neg))
    ok = [(x >= threshold) == (y == 1) for x, y in zip(flat_p, flat_t)]
    out["accuracy"] = sum(ok) / len(ok)
    if pos:
        out["pos_accuracy"] = sum(o for o, y in zip(ok, flat_t) if y == 1) / len(pos)
    if neg:
        out["neg_accuracy"] = sum(o for o, y in zip(ok, flat_t) if y == 0) / len(neg)
    return out
