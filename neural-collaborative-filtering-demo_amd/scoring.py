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
select pipeline (``GraphedScorer``: the same pipeline captured once as a hipGraph and replayed);
``sharded_score_topk`` is the item-sharded multi-GPU form: every
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
QD = 64   # the scan's row width (ncf_score_queries pads narrower rows to it)


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
        if D not in (16, 32, 64, 128):
            # (the scan kernels are 64 deep: narrower rows are zero-padded to 64, which leaves
            # every dot product the D-term one; D = 128 — the C4 model — takes the fp32 scan's
            # 128-deep form, k_collect<128>, with the fp32 threshold sample)
            raise NotImplementedError("the scoring kernels take D = 16, 32, 64 or 128")
        qd = max(QD, D)
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
        self.dim = D
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        pD = torch.empty(I, D, device=dev)
        _lib.call("ncf_gather_rows", ptr(ids), I, ptr(table), model.num_products, D,
                  ptr(model.mf_norm.weight),
                  ptr(model.mf_norm.bias), LN_EPS, ptr(pD), ptr(err), st)
        if D == qd:
            self.p = pD
        else:   # zero-padded to the scan's 64-deep rows (the queries are padded alike)
            self.p = torch.zeros(I, qd, device=dev)
            self.p[:, :D].copy_(pD)
            del pD
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
        # the item rows as three bf16 planes for the split-operand MFMA scan (fp32 accuracy)
        self.p3 = None
        self.pmax = None   # max_i |p_i| (float bits) for the 1/2-term scan's threshold margin
        self.terms = SPLIT_TERMS   # operand terms of the split scan (with pmax; else 3)
        if SPLIT_SCAN and qd == QD:    # (the split planes and their scan are 64 deep)
            self.p3 = torch.empty(3, I, QD, dtype=torch.int16, device=dev)
            _lib.call("ncf_score_split_items", ptr(self.p), I, QD, ptr(self.p3), st)
            if SPLIT_TERMS < 3:
                self.pmax = torch.empty(1, dtype=torch.int32, device=dev)
                _lib.call("ncf_score_item_norm_max", ptr(self.p), I, QD, ptr(self.pmax), st)
        self.version = _param_version(model)

    def valid_for(self, model) -> bool:
        return model is self.model and self.version == _param_version(model)


def _param_version(model):
    # torch's _version sees optimizer steps through torch; engine.updates the HIP kernels' writes
    return (model._engine.updates,) + tuple(p._version for p in model.parameters())


# the candidate scan on bf16 matrix cores with split operands (fp32 accuracy, same candidate
# sets; an index without the planes, p3 = None, takes the fp32 MFMA scan)
SPLIT_SCAN = True
# terms per operand of the split scan: 1 (one bf16 product per pair) or 2 (three products) — the
# thresholds lowered by the scan's error bound, the candidates near the K-th re-scored in fp32, so
# the top-k are the same bits either way (tested) — or 3 (six products, fp32-accurate logits
# straight from the scan).  Measured (10K users x 1M items, ms, top-10 / top-100): 1 term
# 2.85 / 4.29 (scan 2.06 / 2.42), 2 terms 4.75 / 5.76 (scan 3.67 / 3.82), 3 terms 6.8 / 8.5
SPLIT_TERMS = 1
# >= the scan's |logit error| / (|q|_2 max_i |p_i|_2) (Cauchy-Schwarz over the per-term errors),
# with the fp32 accumulation and the fp32 re-scoring's own rounding: two terms (the dropped
# products ~2^-16 relative): ~6.1e-5; one term (bf16 keeps 8 significant bits: each operand
# rounded within 2^-8 of itself, |a0 b0 - a b| <= (2^-7 + 2^-16) |a| |b|): 7.83e-3 + 2 x 64 x
# 2^-24 = 7.84e-3
MARGIN_C = {1: 8e-3, 2: 1e-4}


def _terms(idx):
    return idx.terms if idx.pmax is not None else 3


def _collect(idx, q, rows, n, thr, cap, count, cand, st, expected=0, terms=None):
    """ncf_score_collect(_split) of n queried users over the index's items (``expected``: the
    candidates per user the thresholds aim at, which sizes the split scan's item split;
    ``terms``: the split scan's operand terms, default the index's)."""
    I, D = idx.p.shape
    if idx.p3 is not None:
        terms = terms or _terms(idx)
        if terms < 3:   # lower the thresholds by the scan's error bound first
            _lib.call("ncf_score_margin", q, rows, n, D, ptr(idx.pmax), MARGIN_C[terms], thr, st)
        _lib.call("ncf_score_collect_split", q, rows, n, ptr(idx.p3), ptr(idx.bias), I, D, thr,
                  cap, count, cand, terms, int(expected), st)
    else:
        _lib.call("ncf_score_collect", q, rows, n, ptr(idx.p), ptr(idx.bias), I, D, thr, cap,
                  count, cand, st)


# Expected candidates per user the threshold sample aims at: 512 (a bigger sample costs a
# longer sample GEMM and k-th select, a smaller one more scan hits and select work; round 1,
# fp32 scan: 1024 -> 7.5 ms, 2048 -> 7.7, cap / 2 = 4096 -> 8.3 at top-10 over 1M items), with the sample
# kept within the k-th kernel's LDS-resident size (top-100: ~2570; a 30720-logit cap: 6.26 ms,
# 38912: 5.90 ms), and never above cap / 2.
# (round 4, 10K x 1M eager, 2-4 interleaved runs: top-10 2.61-2.64 ms at 512 (scan 1.78-1.80,
# sample + k-th 0.42) against 2.64-2.82 at 1024 (scan 1.99-2.04, sample + k-th 0.21) and
# 2.99-3.16 at 2048; top-100 takes the rank-j plan, unaffected)
SAMPLE_CANDS = 512
# the collect scans its users in threshold order (see _TopKRun.launch).  Off: measured slower
# (graphed top-10 2.21 / 2.23 against 2.15 / 2.16 ms, r5zk: the scan no faster — the thresholds
# of a user block are already close — and the sort on top)
SORT_USERS = False
# the split scan's item split raised from the expected candidates per user (the launch's
# expected_per_user: fewer per-wave LDS slice overflows; tested invisible in the results)
SIZED_SPLIT = True
KTH_LDS_MAX = 38912   # = score.hip kKthLdsMax
# the threshold sample on bf16 matrix cores, fp16 logits rounded down (ncf_score_sample_split16 +
# ncf_score_kth16, its k-th lowered by the two-term bound) instead of the fp32 sample GEMM +
# fp32 k-th (measured, 10K x 1M eager: top-100 4.25 -> 3.73 ms, top-10 2.78 -> 2.70); needs the
# split index (p3, pmax); tests compare both
SAMPLE16 = True
# the fp16 sample keeps only the maximum of every SAMPLE_GROUP consecutive sample items (the k-th
# largest group maximum bounds the k-th largest logit from below as well), where the sample
# holds >= 8 j group maxima: 8x fewer bytes written and selected over; 1 = every logit
SAMPLE_GROUP = 8


def _select(idx, rows, n, run, k, out_s, out_i, overflow, st, terms=None, check=None):
    """ncf_score_select(_rescored) of n users' candidate lists (fp32 re-scoring after a one- or
    two-term scan; ``terms`` as the scan's; ``check``: the rank-j thresholds to verify the
    selection against, flag 2 where it is not provably the top k)."""
    if idx.pmax is not None:
        _lib.call("ncf_score_select_rescored", rows, n, ptr(run.count), ptr(run.cand), run.cap, k, ptr(run.q), ptr(idx.p), ptr(idx.bias),
                  idx.p.shape[1], ptr(idx.pmax), MARGIN_C[terms or _terms(idx)], out_s, out_i,
                  ptr(run.thr), overflow, check, st)
    else:
        _lib.call("ncf_score_select", rows, n, ptr(run.count), ptr(run.cand), run.cap, k, out_s, out_i, ptr(run.thr), overflow, st)


# Rank-j thresholds (the fp16 sample path, k > RANK_J): the threshold is the sample's j-th
# largest logit (j = RANK_J) instead of its k-th, over a sample k / j times smaller, aimed at
# RANK_J * k expected candidates per user.  It is not a guaranteed bound of the k-th logit, so the
# select verifies each user's result against it (every item at or above it was collected; the
# k chosen are exact iff k were found and the k-th is at or above it) and flags the rest, which
# are re-run from the sample's k-th (guaranteed).  The number of items at or above the j-th of a
# sample of S ~ n_items / k is ~ Gamma(j) * k: below k with probability P(Gamma(16) < 1) ~ 1e-14
# per user on exchangeable scores.  RANK_J = 0: the k-th always.
RANK_J = 16
SAMPLE_MIN = 4096   # items in the smallest threshold sample
# Rank-j sample size factor f: S ~ f n_items / k, so ~RANK_J k / f candidates per user are
# expected and a user needs the guaranteed re-run with probability P(Gamma(RANK_J) < f)
# (f = 2: ~4e-10 per user).  Measured at top-100 (10K x 1M, graphed): f = 1 2.62 / 2.68 ms, f = 2
# 3.29 / 3.33, f = 3 3.28 / 3.41 (r5zl: the larger samples' scans were slower, not faster)
RANK_SAMPLE_F = 1


def _threshold_rank(k: int, cap: int, s16: bool) -> int:
    """The sample rank whose logit is the collect threshold: k, or RANK_J (see above)."""
    if s16 and RANK_J > 0 and k > RANK_J and RANK_J * k <= cap // 2:
        return RANK_J
    return k


def _sample_size(n_items: int, k: int, cap: int, j: int = 0) -> int:
    """Items in the threshold sample S: expected candidates ~ j * n_items / S (j = k by
    default; j < k: the rank-j plan, S ~ n_items / k, RANK_J * k candidates expected)."""
    j = j or k
    if j < k:
        s = max(SAMPLE_MIN, -(-j * n_items * RANK_SAMPLE_F // (RANK_J * k)))
    else:
        s = max(SAMPLE_MIN, -(-k * n_items // max(1, SAMPLE_CANDS)))
    s = max(min(s, KTH_LDS_MAX), -(-2 * j * n_items // cap))
    s = -(-s // 256) * 256
    return min(n_items, s)


class _TopKRun:
    """Buffers and launch sequence of one top-k pipeline for ``n`` users (shared by the eager
    ``score_topk`` and the captured ``GraphedScorer``)."""

    def __init__(self, index: "ItemIndex", n: int, k: int, cap: int):
        p = index.p
        dev = p.device
        I, D = p.shape
        if not 1 <= k <= min(I, cap):
            raise ValueError(f"k must be in [1, {min(I, cap)}]")
        self.index, self.n, self.k, self.cap = index, n, k, cap
        s16 = SAMPLE16 and index.p3 is not None and index.pmax is not None
        self.j = _threshold_rank(k, cap, s16)
        self.S = _sample_size(I, k, cap, self.j)
        self.stride = I // self.S
        # the sample's item biases, contiguous: added in the sample GEMM's epilogue
        self.sbias = index.bias[::self.stride][:self.S].contiguous()
        e = lambda *sh, dt=torch.float32: torch.empty(*sh, dtype=dt, device=dev)  # noqa: E731
        self.uid = e(max(n, 1), dt=torch.int64)
        self.s16 = s16 and self.S <= KTH_LDS_MAX
        # (rank j only where the sample leaves >= 8 k candidates expected: a small catalogue's
        # sample floor of 4096 items would otherwise put the j-th near the k-th item overall)
        if self.j < k and (not self.s16 or self.j * I < 8 * k * self.S):
            self.j = k
            self.S = _sample_size(I, k, cap)
            self.stride = I // self.S
            self.sbias = index.bias[::self.stride][:self.S].contiguous()
        # sample group maxima (fp16 path): rows of Sg = ceil(S / G)
        self.G = SAMPLE_GROUP if self.s16 and SAMPLE_GROUP > 1 and \
            self.S // SAMPLE_GROUP >= 8 * self.j else 1
        self.Sg = -(-self.S // self.G)
        self.q, self.thr = e(max(n, 1), D), e(max(n, 1))
        # the rank-j thresholds before the margins (the select's check)
        self.thr_chk = e(max(n, 1)) if self.j < k else None
        self.sample = (torch.empty(max(n, 1), self.Sg, dtype=torch.int16, device=dev) if self.s16
                       else e(max(n, 1), self.S))
        self.count = torch.zeros(max(n, 1), dtype=torch.int32, device=dev)
        # (logit f32, item i32) records, ncf_score_cand: one 8-byte store per candidate
        self.cand = e(max(n, 1), cap, 2, dt=torch.int32)
        self.overflow = e(max(n, 1), dt=torch.int32)
        self.scores, self.items = e(n, k), e(n, k, dt=torch.int64)
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)

    def launch(self, model, st):
        """queries -> threshold sample (MFMA GEMM over strided item rows) -> k-th threshold ->
        MFMA collect -> select, on stream ``st``; reads self.uid[:n]."""
        idx, n, k, cap = self.index, self.n, self.k, self.cap
        p, bias = idx.p, idx.bias
        I, D = p.shape
        table = model.mf_embedding_collection.embedding_bags["user_id"].weight
        _lib.call("ncf_score_queries", ptr(self.uid), n, ptr(table), model.num_users,
                  model.mf_embedding_dim,
                  ptr(model.mf_norm.weight), ptr(model.mf_norm.bias), LN_EPS,
                  ptr(model.mf_output.weight), ptr(model.final[0].weight), ptr(self.q),
                  ptr(self.err), st)
        if self.s16:
            _lib.call("ncf_score_sample_split16", ptr(self.q), n, ptr(idx.p3), I, D, self.stride,
                      ptr(self.sbias), self.S, self.G, ptr(self.sample), st)
            _lib.call("ncf_score_kth16", ptr(self.sample), n, self.Sg, self.j, ptr(self.thr), st)
            if self.thr_chk is not None:
                self.thr_chk.copy_(self.thr)
            # (the k-th of the fp16 sample is a bound after the two-term error is taken off)
            _lib.call("ncf_score_margin", ptr(self.q), None, n, D, ptr(idx.pmax), MARGIN_C[2],
                      ptr(self.thr), st)
        else:
            _lib.call("ncf_gemm_f32", n, self.S, D, ptr(self.q), D, 0, ptr(p), D * self.stride, 1,
                      ptr(self.sample), self.S, ptr(self.sbias), 0, st)
            _lib.call("ncf_score_kth", ptr(self.sample), n, self.S, k, None, self.stride,
                      ptr(self.thr), st)
        self.count.zero_()
        # the scan's users in threshold order (SORT_USERS): its 32-user blocks then hold users of
        # near-equal thresholds, so its first reject (a lane's best logit against the smallest
        # of its 16 users' thresholds) is nearly as tight as the per-user test
        rows = None
        if SORT_USERS and n >= 64:
            self.order = torch.argsort(self.thr[:n]).to(torch.int32)
            rows = ptr(self.order)
        # expected candidates per user: k x I / S (the threshold sample's k-th over S items)
        _collect(idx, ptr(self.q), rows, n, ptr(self.thr), cap, ptr(self.count), ptr(self.cand),
                 st, expected=-(-self.j * I // self.S) if SIZED_SPLIT else 0)
        _select(idx, None, n, self, k, ptr(self.scores), ptr(self.items), ptr(self.overflow), st,
                check=None if self.thr_chk is None else ptr(self.thr_chk))

    def safe_thresholds(self, redo, st):
        """Users flagged by the rank-j check: their threshold from the sample's k-th instead (the
        fp32 sample GEMM over the same strided items, its k-th: k sample items at or above it, a
        guaranteed bound; the re-run's collect lowers it by the scan's margin)."""
        idx, k = self.index, self.k
        p = idx.p
        I, D = p.shape
        q = self.q[redo].contiguous()
        nr = q.shape[0]
        # (a sample sized for the k-th itself, ~k I / S candidates within cap: the rank-j
        # sample's S ~ I / k would expect ~k^2 of them, over the cap at k = 100, and cost every
        # flagged user a further overflow round)
        S = _sample_size(I, k, self.cap)
        stride = I // S
        sbias = idx.bias[::stride][:S].contiguous()
        sample = torch.empty(nr, S, device=p.device)
        thr = torch.empty(nr, device=p.device)
        _lib.call("ncf_gemm_f32", nr, S, D, ptr(q), D, 0, ptr(p), D * stride, 1,
                  ptr(sample), S, ptr(sbias), 0, st)
        _lib.call("ncf_score_kth", ptr(sample), nr, S, k, None, stride, ptr(thr), st)
        self.thr[redo] = thr

    def redo_overflow(self, st):
        """Re-run the users whose candidate list overflowed (flag 1) or whose rank-j result was
        not provably exact (flag 2) (eager; rare: the threshold sample targets cap / 2
        candidates at most, and a rank-j shortfall has probability ~1e-14 per user)."""
        idx, k, cap = self.index, self.k, self.cap
        p, bias = idx.p, idx.bias
        I, D = p.shape
        dev = p.device
        overflow = self.overflow[:self.n]
        # the re-runs scan with at least two terms: their thresholds (the K-th re-scored logit
        # seen) sit just below the K-th, and the one-term scan's margin (~8e-3 |q| max|p|) could
        # keep more than cap items above the lowered threshold
        terms = max(2, _terms(idx))
        for _ in range(32):
            redo = torch.nonzero(overflow).flatten()
            if redo.numel() == 0:
                return
            short = redo[overflow[redo] == 2]
            if short.numel():
                self.safe_thresholds(short, st)
            rows = redo.to(torch.int32)
            self.count[redo] = 0
            sub_s = torch.empty(rows.numel(), k, device=dev)
            sub_i = torch.empty(rows.numel(), k, dtype=torch.int64, device=dev)
            sub_o = torch.empty(rows.numel(), dtype=torch.int32, device=dev)
            _collect(idx, ptr(self.q), ptr(rows), rows.numel(), ptr(self.thr), cap,
                     ptr(self.count), ptr(self.cand), st, terms=terms)
            _select(idx, ptr(rows), rows.numel(), self, k, ptr(sub_s), ptr(sub_i), ptr(sub_o), st,
                    terms=terms)
            self.scores[redo] = sub_s
            self.items[redo] = sub_i
            overflow.zero_()
            overflow[redo] = sub_o
        raise RuntimeError("score_topk: candidate lists kept overflowing (degenerate scores?)")

    def result(self):
        items = self.items
        if self.index.ids is not None:   # shard-local positions -> global item ids
            items = self.index.ids[items.clamp_min(0)]
        return self.scores, items


def score_topk(model, user_ids: torch.Tensor, k: int = 10, index: Optional[ItemIndex] = None,
               cap: int = 8192) -> Tuple[torch.Tensor, torch.Tensor]:
    """Top-k (probability, item id) per user over all items, as
    ``forward_simple(user, all_items)`` + ``nlargest(k)`` would rank them.  Returns
    ``(scores [n, k] fp32, items [n, k] int64)``."""
    if index is None:
        index = ItemIndex(model)
    elif not index.valid_for(model):   # parameters changed since the index was built
        index = ItemIndex(model, items=index.ids)
    dev = index.p.device
    uid = user_ids.to(device=dev, dtype=torch.int64).contiguous()
    n = uid.numel()
    run = _TopKRun(index, n, k, cap)
    if n == 0:
        return run.result()
    st = _lib.stream_ptr(dev)
    run.uid[:n].copy_(uid)
    run.launch(model, st)
    run.redo_overflow(st)
    if int(run.err.item()):
        raise IndexError("score_topk: user id out of range of the embedding table")
    return run.result()


class GraphedScorer:
    """C5 as a captured hipGraph (BASELINE configs[4]): the whole top-k pipeline for a fixed
    number of users (queries, threshold sample GEMM, k-th threshold, MFMA collect, select, and
    the overflow / id-error flags) recorded once with ``torch.cuda.CUDAGraph`` and replayed per
    call, so a call costs one graph launch and one 8-byte flag read instead of the per-launch
    host work.  Users whose candidate list overflowed are re-run eagerly (same results as
    ``score_topk``); a parameter change since capture rebuilds the index and re-captures.

        scorer = GraphedScorer(model, n_users=10_000, k=10)
        scores, items = scorer(user_ids)        # [n, k] each, like score_topk

    The graph writes into static output tensors.  By default a call returns fresh copies of
    them (like ``score_topk``); ``scorer(user_ids, copy=False)`` returns the static tensors
    themselves, which the NEXT call overwrites in place.
    """

    def __init__(self, model, n_users: int, k: int = 10, index: Optional[ItemIndex] = None,
                 cap: int = 8192):
        self.model, self.n, self.k, self.cap = model, int(n_users), int(k), cap
        if self.n < 1:
            raise ValueError("GraphedScorer needs n_users >= 1")
        self.index = index if index is not None and index.valid_for(model) else ItemIndex(
            model, items=None if index is None else index.ids)
        self._capture()

    def _capture(self):
        idx = self.index
        dev = idx.p.device
        self.run = run = _TopKRun(idx, self.n, self.k, self.cap)
        run.uid.zero_()
        st = _lib.stream_ptr(dev)
        run.launch(self.model, st)           # warm-up: kernel attributes, lazy module loads
        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph()
        # thread_local: other threads' HIP calls (e.g. a process group's watchdog polling its
        # events) stay legal while this thread captures
        with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
            run.launch(self.model, _lib.stream_ptr(dev))
            self.flags = torch.stack([run.overflow[:self.n].amax(), run.err[0]])
            self.out = run.result()
        self.version = idx.version

    def __call__(self, user_ids: torch.Tensor,
                 copy: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
        if not self.index.valid_for(self.model):
            self.index = ItemIndex(self.model, items=self.index.ids)
            self._capture()
        run = self.run
        uid = user_ids.reshape(-1)
        if uid.numel() != self.n:
            raise ValueError(f"GraphedScorer was captured for {self.n} users, got {uid.numel()}")
        run.uid.copy_(uid)
        run.err.zero_()
        self.graph.replay()
        over, err = self.flags.tolist()
        if err:
            raise IndexError("score_topk: user id out of range of the embedding table")
        if over:
            run.redo_overflow(_lib.stream_ptr(run.uid.device))
            out = run.result()
        else:
            out = self.out
        return (out[0].clone(), out[1].clone()) if copy else out


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
                       local_topk=None, merge=None, graph: bool = False):
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
            if graph:   # the shard's pipeline as a captured hipGraph (cached on the index)
                gs = index.__dict__.setdefault("_graphed", {})
                sc = gs.get((u.numel(), kk, cap))
                if sc is None:
                    sc = gs[(u.numel(), kk, cap)] = GraphedScorer(model, u.numel(), kk, index, cap)
                s, i = sc(u)
            else:
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
