"""Standalone HIP ops for the modules that also exist outside the fused AdvancedNCF step:
MultiHeadAttention (any group length <= 64), TemporalEncoding and CategoryHierarchy.

They mirror the reference modules' forward semantics (src/model/architecture.py:35-57, :86-94,
:111-119) and run on the same kernels as the engine (MFMA projections + attention core), with
autograd support for MultiHeadAttention and TemporalEncoding.  GPU only.
"""
import torch

from . import _lib
from ._lib import ptr
from .engine import LN_EPS
from .sparse import gather_rows


def _require_cuda(t):
    if not t.is_cuda:
        raise RuntimeError("ncf_amd ops run on the MI355X only (no CPU fallback)")


def _gemm(A, lda, a_t, B, ldb, b_t, C, ldc, M, N, K, bias=None, accum=False):
    _lib.call("ncf_gemm_direct", M, N, K, ptr(A), lda, int(a_t), ptr(B), ldb, int(b_t), ptr(C), ldc,
              ptr(bias), 2 if accum else 0, _lib.stream_ptr(C.device))


def _wgrad(dY, X, dW, n, m_out, k_in, dbias=None):
    s = max(1, min(160, (n + 127) // 128))
    ws = torch.empty(_lib.query("ncf_gemm_splitk_workspace", m_out, k_in, s), device=dY.device)
    _lib.call("ncf_gemm_f32_splitk", m_out, k_in, n, ptr(dY), m_out, 1, ptr(X), k_in, 0, ptr(dW),
              k_in, 0, ptr(dbias), s, ptr(ws), ws.numel(), None, _lib.stream_ptr(dY.device))


class _MHAFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mod, drop_p, seed, mask, q_in, k_in, v_in, wq, bq, wk, bk, wv, bv, wo, bo):
        Bn, L, D = q_in.shape
        H = mod.num_heads
        n = Bn * L
        dev = q_in.device
        xq, xk, xv = (t.reshape(n, D).contiguous().float() for t in (q_in, k_in, v_in))
        q, k, v, o, y = (torch.empty(n, D, device=dev) for _ in range(5))
        P = torch.empty(Bn * H * L * L, device=dev)
        _gemm(xq, D, 0, wq, D, 1, q, D, n, D, D, bq)
        _gemm(xk, D, 0, wk, D, 1, k, D, n, D, D, bk)
        _gemm(xv, D, 0, wv, D, 1, v, D, n, D, D, bv)
        if mask is None:
            _lib.call("ncf_attention_fwd", ptr(q), ptr(k), ptr(v), Bn, L, H, D, drop_p, seed, None,
                      ptr(P), ptr(o), _lib.stream_ptr(dev))
        else:    # [Bn, H, L, L] bytes, 0 = masked (architecture.py:47-48)
            _lib.call("ncf_attention_fwd_masked", ptr(q), ptr(k), ptr(v), Bn, L, H, D, drop_p, seed,
                      None, ptr(mask), ptr(P), ptr(o), _lib.stream_ptr(dev))
        _gemm(o, D, 0, wo, D, 1, y, D, n, D, D, bo)
        ctx.save_for_backward(xq, xk, xv, q, k, v, P, o, wq, wk, wv, wo)
        ctx.meta = (Bn, L, D, H, drop_p, seed)
        return y.view(Bn, L, D)

    @staticmethod
    def backward(ctx, gy):
        xq, xk, xv, q, k, v, P, o, wq, wk, wv, wo = ctx.saved_tensors
        Bn, L, D, H, drop_p, seed = ctx.meta
        n = Bn * L
        dev = gy.device
        dy = gy.reshape(n, D).contiguous().float()
        g = {nm: torch.empty(D, D, device=dev) for nm in ("wq", "wk", "wv", "wo")}
        gb = {nm: torch.empty(D, device=dev) for nm in ("bq", "bk", "bv", "bo")}
        _wgrad(dy, o, g["wo"], n, D, D, gb["bo"])
        do = torch.empty(n, D, device=dev)
        _gemm(dy, D, 0, wo, D, 0, do, D, n, D, D)
        dS = torch.empty(Bn * H * L * L, device=dev)
        dq, dk, dv = (torch.empty(n, D, device=dev) for _ in range(3))
        _lib.call("ncf_attention_bwd", ptr(q), ptr(k), ptr(v), ptr(P), ptr(do), Bn, L, H, D,
                  drop_p, seed, None, ptr(dS), ptr(dq), ptr(dk), ptr(dv), _lib.stream_ptr(dev))
        outs = []
        for dX, X, W, wn, bn in ((dq, xq, wq, "wq", "bq"), (dk, xk, wk, "wk", "bk"),
                                 (dv, xv, wv, "wv", "bv")):
            _wgrad(dX, X, g[wn], n, D, D, gb[bn])
            gx = torch.empty(n, D, device=dev)
            _gemm(dX, D, 0, W, D, 0, gx, D, n, D, D)
            outs.append(gx.view(Bn, L, D))
        return (None, None, None, None, outs[0], outs[1], outs[2], g["wq"], gb["bq"], g["wk"], gb["bk"],
                g["wv"], gb["bv"], g["wo"], gb["bo"])


def mha_forward(mod, query, key, value, mask=None):
    """MultiHeadAttention.forward (architecture.py:35-57): query/key/value [B, L, D] (a 2-D
    [B, D] input is a length-1 sequence, as the reference's .view(batch, -1, H, hd) makes it).
    ``mask`` (:36, :47-48): any tensor that broadcasts against the scores [B, H, L, L]; where it
    is 0 the score is -inf before the softmax (ncf_attention_fwd_masked)."""
    _require_cuda(query)
    squeeze = query.dim() == 2
    if squeeze:
        query, key, value = query.unsqueeze(1), key.unsqueeze(1), value.unsqueeze(1)
    if key.shape[1] != query.shape[1] or value.shape[1] != key.shape[1]:
        raise NotImplementedError("MultiHeadAttention: key/value length must equal the query's "
                                  "on this path (every reference call site passes equal lengths)")
    drop_p = float(mod.dropout.p) if mod.training else 0.0
    seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if drop_p > 0 else 0
    m8 = None
    if mask is not None:
        Bn, L = query.shape[0], query.shape[1]
        m = torch.as_tensor(mask, device=query.device)
        # masked_fill(mask == 0, .) broadcasts the mask against the scores [B, H, L, L]
        m8 = torch.broadcast_to(m != 0, (Bn, mod.num_heads, L, L)).to(torch.uint8).contiguous()
    y = _MHAFunction.apply(mod, drop_p, seed, m8, query, key, value, mod.q_proj.weight, mod.q_proj.bias,
                           mod.k_proj.weight, mod.k_proj.bias, mod.v_proj.weight, mod.v_proj.bias,
                           mod.out_proj.weight, mod.out_proj.bias)
    return y  # a 2-D input comes back [B, 1, D], as the reference's .view(batch, -1, D) makes it


class _TemporalFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mod, hour, day, month, days_since, wh, wd, wm):
        dev = wh.device
        n = hour.numel()
        T = mod.embed_dim
        ids = [t.reshape(-1).to(device=dev, dtype=torch.int64).contiguous()
               for t in (hour, day, month, days_since)]
        out = torch.empty(n, T, device=dev)
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        _lib.call("ncf_temporal_fwd", *[ptr(t) for t in ids], n, ptr(wh), ptr(wd), ptr(wm),
                  ptr(mod.pe), mod.max_period, T, ptr(out), ptr(err), _lib.stream_ptr(dev))
        if int(err.item()):
            raise IndexError("TemporalEncoding: hour/day/month index out of range")
        ctx.save_for_backward(*ids[:3])
        ctx.T = T
        return out.view(*hour.shape, T)

    @staticmethod
    def backward(ctx, gy):
        h, d, m = ctx.saved_tensors
        T = ctx.T
        dev = gy.device
        gh, gd, gm = torch.empty(24, T, device=dev), torch.empty(7, T, device=dev), torch.empty(12, T, device=dev)
        g = gy.reshape(-1, T).contiguous().float()
        _lib.call("ncf_temporal_bwd", ptr(h), ptr(d), ptr(m), h.numel(), ptr(g), T, ptr(gh), ptr(gd),
                  ptr(gm), _lib.stream_ptr(dev))
        return None, None, None, None, None, gh, gd, gm


def temporal_encoding_forward(mod, hour, day, month, days_since):
    _require_cuda(mod.hour_embed.weight)
    return _TemporalFunction.apply(mod, hour, day, month, days_since, mod.hour_embed.weight,
                                   mod.day_embed.weight, mod.month_embed.weight)


def category_hierarchy_forward(mod, department_ids, category_ids):
    """CategoryHierarchy.forward (architecture.py:111-119) for 1-D id vectors of length n.

    The attention sees one key per query (the reference views the 2-D [n, D] inputs as n
    sequences of length 1), so softmax == 1 and attn = out_proj(v_proj(dept)) with shape
    [n, 1, D].  The residual ``attn + cat_embeds`` then BROADCASTS [n, 1, D] + [n, D] ->
    [n, n, D] (element [a, b] = attn[a] + cat[b]); LayerNorm keeps that shape.  This is the
    reference's behaviour (pinned by F5) and is reproduced exactly.  Inference path
    (get_product_embeddings)."""
    w = mod.department_embed.weight
    _require_cuda(w)
    if torch.is_grad_enabled() and w.requires_grad:
        with torch.no_grad():
            return category_hierarchy_forward(mod, department_ids, category_ids)
    p_attn = float(mod.hierarchy_attn.dropout.p) if mod.training else 0.0
    p_out = float(mod.dropout.p) if mod.training else 0.0
    if p_attn > 0 or p_out > 0:
        return _category_hierarchy_train(mod, department_ids, category_ids, p_attn, p_out)
    dev = w.device
    dept_ids = department_ids.reshape(-1).to(device=dev, dtype=torch.int64)
    cat_ids = category_ids.reshape(-1).to(device=dev, dtype=torch.int64)
    n = dept_ids.numel()
    dept = gather_rows(w, dept_ids)
    D = dept.shape[1]
    att = mod.hierarchy_attn
    v = torch.empty(n, D, device=dev)
    _gemm(dept, D, 0, att.v_proj.weight, D, 1, v, D, n, D, D, att.v_proj.bias)
    a_idx = torch.arange(n, device=dev).repeat_interleave(n)      # row a*n+b <- attn[a]
    b_idx = cat_ids.repeat(n)                                      #            + cat[b]
    vrep = gather_rows(v, a_idx)
    h = gather_rows(mod.category_embed.weight, b_idx)
    _gemm(vrep, D, 0, att.out_proj.weight, D, 1, h, D, n * n, D, D, att.out_proj.bias, accum=True)
    out = torch.empty(n * n, D, device=dev)
    mean, rstd = torch.empty(n * n, device=dev), torch.empty(n * n, device=dev)
    _lib.call("ncf_relu_ln_dropout_fwd", ptr(h), n * n, D, ptr(mod.norm.weight), ptr(mod.norm.bias),
              LN_EPS, 0.0, 0, None, ptr(out), ptr(mean), ptr(rstd), _lib.stream_ptr(dev))
    return out.view(n, n, D)


def _category_hierarchy_train(mod, department_ids, category_ids, p_attn, p_out, seed=None,
                              scales=None):
    """CategoryHierarchy.forward in training mode (architecture.py:111-119 with its dropouts
    active): the attention over one key has weight 1, which the attention's nn.Dropout (:51)
    keeps (x 1/(1-p)) or drops per (row, head); out_proj; the module's nn.Dropout (:117) per
    element; then the broadcast residual + LayerNorm of the eval path.  Masks come from the
    package's dropout stream (`seed`, fresh per call like forward()'s); ``scales`` (a dict) receives
    the keep-scales ("attn" [n, H], "out" [n, D]) for tests.  No autograd (as the eval path)."""
    w = mod.department_embed.weight
    dev = w.device
    dept_ids = department_ids.reshape(-1).to(device=dev, dtype=torch.int64)
    cat_ids = category_ids.reshape(-1).to(device=dev, dtype=torch.int64)
    n = dept_ids.numel()
    att = mod.hierarchy_attn
    D = w.shape[1]
    H = att.num_heads
    if seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    st = _lib.stream_ptr(dev)
    dept = gather_rows(w, dept_ids)
    v = torch.empty(n, D, device=dev)
    _gemm(dept, D, 0, att.v_proj.weight, D, 1, v, D, n, D, D, att.v_proj.bias)
    sa = torch.empty(n, H, device=dev) if scales is not None else None
    _lib.call("ncf_dropout_rows", ptr(v), n, D, D // H, p_attn, seed, ptr(v), ptr(sa), st)
    a = torch.empty(n, D, device=dev)
    _gemm(v, D, 0, att.out_proj.weight, D, 1, a, D, n, D, D, att.out_proj.bias)
    so = torch.empty(n, D, device=dev) if scales is not None else None
    _lib.call("ncf_dropout_rows", ptr(a), n, D, 1, p_out, seed ^ 0x5DEECE66D, ptr(a), ptr(so), st)
    if scales is not None:
        scales["attn"], scales["out"] = sa, so
    a_idx = torch.arange(n, device=dev).repeat_interleave(n)      # row a*n+b <- a[a] + cat[b]
    h = gather_rows(mod.category_embed.weight, cat_ids.repeat(n))
    h += gather_rows(a, a_idx)
    out = torch.empty(n * n, D, device=dev)
    mean, rstd = torch.empty(n * n, device=dev), torch.empty(n * n, device=dev)
    _lib.call("ncf_relu_ln_dropout_fwd", ptr(h), n * n, D, ptr(mod.norm.weight), ptr(mod.norm.bias),
              LN_EPS, 0.0, 0, None, ptr(out), ptr(mean), ptr(rstd), st)
    return out.view(n, n, D)


def forward_simple_hour(model, user_ids, product_ids, hour, projection=None, seed=None):
    """AdvancedNCF.forward_simple(user_ids, product_ids, hour) (architecture.py:409-485).

    te = hour_E[hour] (TemporalEncoding.hour_embed, :434); when temporal_dim != D the reference
    projects it with a FRESH randomly initialised nn.Linear(T, D) on every call (:436-442) — done
    the same way here (torch's default init on the model's device) unless ``projection`` (an
    nn.Linear or (weight, bias)) is given; both item rows are scaled by (1 + 0.3 * proj) (:444,
    :456-458, fused into the gather kernel) and the MLP input is [attention ‖ te] (:467-468)."""
    eng = model._engine
    dev = eng._check_device()
    m = model
    D, T = m.mlp_embedding_dim, m.temporal_dim
    hour = hour.to(device=dev, dtype=torch.int64).contiguous()
    te = gather_rows(m.temporal_encoding.hour_embed.weight, hour)
    n = te.shape[0]
    if T != m.mf_embedding_dim:
        if projection is None:
            projection = torch.nn.Linear(T, m.mf_embedding_dim, device=dev)
        w_p, b_p = projection if isinstance(projection, tuple) else (projection.weight, projection.bias)
        w_p = w_p.detach().to(device=dev, dtype=torch.float32).contiguous()
        b_p = b_p.detach().to(device=dev, dtype=torch.float32).contiguous()
        tp = torch.empty(n, m.mf_embedding_dim, device=dev)
        _lib.call("ncf_gemm_f32", n, m.mf_embedding_dim, T, ptr(te), T, 0, ptr(w_p), T, 1, ptr(tp),
                  m.mf_embedding_dim, ptr(b_p), 0, _lib.stream_ptr(dev))
    else:
        tp = te
    # training mode (the reference's nn.Dropout layers active, :458-473): the attention's
    # dropout on its single-key weight and the tower's after every LayerNorm, from the package's
    # dropout stream (a fresh seed per call unless given); no backward through this path
    drop_p = float(m.dropout) if m.training else 0.0
    if drop_p > 0 and seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    w = eng.forward(user_ids, product_ids, 1, False, drop_p, seed or 0, temporal=(tp, 0.3, te))
    eng.check_ids(w)
    return w.prob.clone()
