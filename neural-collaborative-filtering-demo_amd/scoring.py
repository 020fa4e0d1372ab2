"""Batch candidate scoring (C5): top-K items per user over the whole catalogue.

The reference serves recommendations with ``model.forward_simple(customer, all_products)`` and
``DataFrame.nlargest(top_k, 'score')`` (src/inference/demo/app.py:44-75).  ``score_topk`` returns
the same top-K (probabilities and item ids, ordered by score desc then item id asc) for many users
at once through the factorised eval form (csrc/score.hip):

    logit(u, i) = q_u . p_i + bias_i
    q_u    = w0 * LN_mf(U_mf[u]) * w_mf                 (ncf_score_queries)
    p_i    = LN_mf(I_mf[i])                              (ncf_gather_rows, cached per model state)
    bias_i = w1 * mlp_item(i) + w0 * b_mf + b_final      (the engine's eval forward + ncf_score_item_bias)

``ItemIndex`` caches the item side (p, bias) for a parameter version (optionally for a subset
of the catalogue: one rank's item shard); ``score_topk`` runs the threshold / MFMA-collect /
select pipeline; ``sharded_score_topk`` is the item-sharded multi-GPU form: every
rank scores all queried users against its own item shard, the per-shard top-K lists are
all-gathered (RCCL) and merged per user by ``ncf_score_merge``.  ``forward_simple(hour=None)`` semantics only (the
hour variant draws a fresh random projection on every call, architecture.py:437-442, so it has no
reusable item side).  GPU only; no CPU fallback.
"""
from typing import Optional, Tuple

import torch

from . import _lib
from ._lib import ptr
from .engine import LN_EPS

K_MF_U = "mf_embedding_collection.embedding_bags.user_id.weight"
K_MF_I = "mf_embedding_collection.embedding_bags.product_id.weight"


class ItemIndex:
    """Item-side factors of the factorised scorer for one model state."""

    def __init__(self, model, chunk: int = 65536, items: Optional[torch.Tensor] = None):
        """``items``: the global item ids this index covers (default: the whole catalogue)."""
        eng = model._engine
        eng.sync_tables()
        self.model = model
        dev = model.mf_norm.weight.device
        if dev.type != "cuda":
            raise RuntimeError("ncf_amd scoring runs on the MI355X only (no CPU fallback)")
        I = model.num_products
        D = model.mf_embedding_dim
        if D != 64 or model.mlp_embedding_dim != 64:
            raise NotImplementedError("the scoring kernels are specialised for D = 64")
        st = _lib.stream_ptr(dev)
        if items is None:
            ids = torch.arange(I, dtype=torch.int64, device=dev)
            self.ids = None
        else:
            ids = items.to(device=dev, dtype=torch.int64).contiguous()
            if ids.numel() and (int(ids.min()) < 0 or int(ids.max()) >= I):
                raise IndexError("ItemIndex: item id out of range of the embedding table")
            self.ids = ids
            I = ids.numel()
        table = model.mf_embedding_collection.embedding_bags["product_id"].weight
        self.p = torch.empty(I, D, device=dev)
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        _lib.call("ncf_gather_rows", ptr(ids), I, ptr(table), model.num_products, D,
                  ptr(model.mf_norm.weight),
                  ptr(model.mf_norm.bias), LN_EPS, ptr(self.p), ptr(err), st)
        # mlp_item(i): the eval forward's MLP prediction depends on the item only (M = 1)
        mlp_item = torch.empty(I, device=dev)
        zeros = torch.zeros(max(1, min(I, chunk)), dtype=torch.int64, device=dev)
        with torch.no_grad():
            for c0 in range(0, I, chunk):
                c1 = min(I, c0 + chunk)
                w = eng.forward(zeros[:c1 - c0], ids[c0:c1], 1, False, 0.0, 0)
                mlp_item[c0:c1].copy_(w.mlp_pred)
        self.bias = torch.empty(I, device=dev)
        _lib.call("ncf_score_item_bias", ptr(mlp_item), I, ptr(model.final[0].weight),
                  ptr(model.final[0].bias), ptr(model.mf_output.bias), ptr(self.bias), st)
        self.version = _param_version(model)

    def valid_for(self, model) -> bool:
        return model is self.model and self.version == _param_version(model)


def _param_version(model):
    # torch's _version sees optimizer steps through torch; engine.updates the HIP kernels' writes
    return (model._engine.updates,) + tuple(p._version for p in model.parameters())


def _sample_size(n_items: int, k: int, cap: int) -> int:
    """Items in the threshold sample: expected candidates ~ k * n_items / S <= cap / 2."""
    s = max(4096, -(-2 * k * n_items // cap))
    s = -(-s // 256) * 256
    return min(n_items, s)


def score_topk(model, user_ids: torch.Tensor, k: int = 10, index: Optional[ItemIndex] = None,
               cap: int = 8192) -> Tuple[torch.Tensor, torch.Tensor]:
    """Top-k (probability, item id) per user over all items, as
    ``forward_simple(user, all_items)`` + ``nlargest(k)`` would rank them.  Returns
    ``(scores [n, k] fp32, items [n, k] int64)``."""
    if index is None:
        index = ItemIndex(model)
    elif not index.valid_for(model):   # parameters changed since the index was built
        index = ItemIndex(model, items=index.ids)
    p, bias = index.p, index.bias
    dev = p.device
    I, D = p.shape
    if not 1 <= k <= min(I, cap):
        raise ValueError(f"k must be in [1, {min(I, cap)}]")
    st = _lib.stream_ptr(dev)
    uid = user_ids.to(device=dev, dtype=torch.int64).contiguous()
    n = uid.numel()
    scores = torch.empty(n, k, device=dev)
    items = torch.empty(n, k, dtype=torch.int64, device=dev)
    if n == 0:
        return scores, items
    # 1. queries
    q = torch.empty(n, D, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    table = model.mf_embedding_collection.embedding_bags["user_id"].weight
    _lib.call("ncf_score_queries", ptr(uid), n, ptr(table), model.num_users, D,
              ptr(model.mf_norm.weight), ptr(model.mf_norm.bias), LN_EPS,
              ptr(model.mf_output.weight), ptr(model.final[0].weight), ptr(q), ptr(err), st)
    # 2. thresholds from a strided sample of items (logits via the MFMA GEMM, strided B rows)
    S = _sample_size(I, k, cap)
    stride = I // S
    sample = torch.empty(n, S, device=dev)
    _lib.call("ncf_gemm_f32", n, S, D, ptr(q), D, 0, ptr(p), D * stride, 1, ptr(sample), S, None,
              0, st)
    thr = torch.empty(n, device=dev)
    _lib.call("ncf_score_kth", ptr(sample), n, S, k, ptr(bias), stride, ptr(thr), st)
    del sample
    # 3./4. collect + select; re-run the users whose candidate list overflowed
    count = torch.zeros(n, dtype=torch.int32, device=dev)
    cand_l = torch.empty(n, cap, device=dev)
    cand_i = torch.empty(n, cap, dtype=torch.int32, device=dev)
    overflow = torch.empty(n, dtype=torch.int32, device=dev)
    _lib.call("ncf_score_collect", ptr(q), None, n, ptr(p), ptr(bias), I, D, ptr(thr), cap,
              ptr(count), ptr(cand_l), ptr(cand_i), st)
    _lib.call("ncf_score_select", None, n, ptr(count), ptr(cand_l), ptr(cand_i), cap, k,
              ptr(scores), ptr(items), ptr(thr), ptr(overflow), st)
    for _ in range(32):
        redo = torch.nonzero(overflow).flatten()
        if redo.numel() == 0:
            break
        rows = redo.to(torch.int32)
        count[redo] = 0
        sub_s = torch.empty(rows.numel(), k, device=dev)
        sub_i = torch.empty(rows.numel(), k, dtype=torch.int64, device=dev)
        sub_o = torch.empty(rows.numel(), dtype=torch.int32, device=dev)
        _lib.call("ncf_score_collect", ptr(q), ptr(rows), rows.numel(), ptr(p), ptr(bias), I, D,
                  ptr(thr), cap, ptr(count), ptr(cand_l), ptr(cand_i), st)
        _lib.call("ncf_score_select", ptr(rows), rows.numel(), ptr(count), ptr(cand_l),
                  ptr(cand_i), cap, k, ptr(sub_s), ptr(sub_i), ptr(thr), ptr(sub_o), st)
        scores[redo] = sub_s
        items[redo] = sub_i
        overflow.zero_()
        overflow[redo] = sub_o
    else:
        raise RuntimeError("score_topk: candidate lists kept overflowing (degenerate scores?)")
    if int(err.item()):
        raise IndexError("score_topk: user id out of range of the embedding table")
    if index.ids is not None:   # shard-local positions -> global item ids
        items = index.ids[items.clamp_min(0)]
    return scores, items


def shard_items(num_items: int, world: int, rank: int) -> torch.Tensor:
    """Global item ids of ``rank``'s scoring shard: a contiguous block of the catalogue."""
    per = -(-num_items // world)
    return torch.arange(min(num_items, rank * per), min(num_items, (rank + 1) * per),
                        dtype=torch.int64)


def merge_topk(cand_scores: torch.Tensor, cand_items: torch.Tensor, k: int):
    """Per-user top-k of ``[n, L]`` candidate (score, global item id) lists, ordered by score
    desc then item id asc (empty slots: id < 0).  HIP (ncf_score_merge); GPU only."""
    if cand_scores.device.type != "cuda":
        raise RuntimeError("ncf_amd scoring runs on the MI355X only (no CPU fallback)")
    n, L = cand_scores.shape
    s = cand_scores.to(torch.float32).contiguous()
    it = cand_items.to(torch.int64).contiguous()
    out_s = torch.empty(n, k, device=s.device)
    out_i = torch.empty(n, k, dtype=torch.int64, device=s.device)
    _lib.call("ncf_score_merge", ptr(s), ptr(it), n, L, k, ptr(out_s), ptr(out_i),
              _lib.stream_ptr(s.device))
    return out_s, out_i


def sharded_score_topk(model, user_ids: torch.Tensor, k: int = 10,
                       index: Optional[ItemIndex] = None, group=None, cap: int = 8192,
                       local_topk=None, merge=None):
    """Item-sharded C5 scoring over ``torch.distributed``: rank r scores every
    queried user against ``shard_items(I, W, r)``, the ``[n, k]`` local lists are all-gathered
    (8 B per entry + id widening) and merged per user.  Every rank returns the global top-k.
    ``local_topk(user_ids, k) -> (scores, global ids)`` and ``merge`` default to the HIP path
    (they are parameters so the collective layout can be exercised on CPU ranks)."""
    import torch.distributed as dist
    W = dist.get_world_size(group) if dist.is_initialized() else 1
    r = dist.get_rank(group) if dist.is_initialized() else 0
    if local_topk is None:
        if index is None or not index.valid_for(model):
            index = ItemIndex(model, items=shard_items(model.num_products, W, r))
        kk = min(k, index.p.shape[0])

        def local_topk(u, _k):
            s, i = score_topk(model, u, kk, index, cap)
            if kk < _k:   # a shard smaller than k: pad with empty slots
                s = torch.cat([s, s.new_zeros(s.shape[0], _k - kk)], 1)
                i = torch.cat([i, i.new_full((i.shape[0], _k - kk), -1)], 1)
            return s, i
    merge = merge or merge_topk
    s, i = local_topk(user_ids, k)
    if W == 1:
        return s, i      # already the (score desc, item id asc) top-k of the whole catalogue
    gs = [torch.empty_like(s) for _ in range(W)]
    gi = [torch.empty_like(i) for _ in range(W)]
    dist.all_gather(gs, s.contiguous(), group=group)
    dist.all_gather(gi, i.contiguous(), group=group)
    return merge(torch.cat(gs, 1), torch.cat(gi, 1), k)
