"""AdvancedNCF — drop-in for src/model/architecture.py of the reference, MI355X-native.

Same constructor, same attribute names, same 62 state_dict keys in the same order, same
forward / forward_simple / get_user_embeddings / get_product_embeddings signatures.  The math
of the hot path runs in the HIP kernels of libncf_hip.so (engine.py); there is no CPU fallback.

Reference citations are src/model/architecture.py:<line> unless stated.
"""
import logging
import math
import weakref
from typing import Dict, List, Optional

import torch
import torch.nn as nn

from . import _lib
from .engine import NCFEngine, LN_EPS
from .sparse import (EmbeddingBagCollection, EmbeddingBagConfig, KeyedJaggedTensor, PoolingType,
                     gather_rows)
from . import optim as _optim

log = logging.getLogger(__name__)


class MultiHeadAttention(nn.Module):
    """Parameter container with the reference's names (:18-33).  Inside AdvancedNCF its math
    runs in the fused engine; standalone use (CategoryHierarchy with L = 1) goes through
    ``attend_single_key``."""

    def __init__(self, embed_dim: int, num_heads: int = 4, dropout: float = 0.1):
        super().__init__()
        assert embed_dim % num_heads == 0, "embed_dim must be divisible by num_heads"
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.head_dim = embed_dim // num_heads
        self.q_proj = nn.Linear(embed_dim, embed_dim)
        self.k_proj = nn.Linear(embed_dim, embed_dim)
        self.v_proj = nn.Linear(embed_dim, embed_dim)
        self.out_proj = nn.Linear(embed_dim, embed_dim)
        self.dropout = nn.Dropout(dropout)
        self.scale = math.sqrt(self.head_dim)

    def forward(self, query, key, value, mask=None):
        from .ops import mha_forward
        return mha_forward(self, query, key, value, mask)


class TemporalEncoding(nn.Module):
    """hour/day/month embeddings + sinusoidal seasonal table (:59-94)."""

    def __init__(self, embed_dim: int, max_period: int = 365):
        super().__init__()
        self.embed_dim = embed_dim
        self.max_period = max_period
        self.hour_embed = nn.Embedding(24, embed_dim)
        self.day_embed = nn.Embedding(7, embed_dim)
        self.month_embed = nn.Embedding(12, embed_dim)
        position = torch.arange(max_period).unsqueeze(1)
        div_term = torch.exp(torch.arange(0, embed_dim, 2) * (-math.log(10000.0) / embed_dim))
        pe = torch.zeros(max_period, embed_dim)
        pe[:, 0::2] = torch.sin(position * div_term)
        pe[:, 1::2] = torch.cos(position * div_term)
        self.register_buffer("pe", pe)

    def forward(self, hour, day, month, days_since):
        from .ops import temporal_encoding_forward
        return temporal_encoding_forward(self, hour, day, month, days_since)


class CategoryHierarchy(nn.Module):
    """department/category embeddings + attention + residual LayerNorm (:96-119)."""

    def __init__(self, num_departments: int, num_categories: int, embed_dim: int,
                 dropout: float = 0.1):
        super().__init__()
        self.department_embed = nn.Embedding(num_departments, embed_dim)
        self.category_embed = nn.Embedding(num_categories, embed_dim)
        self.hierarchy_attn = MultiHeadAttention(embed_dim, num_heads=4, dropout=dropout)
        self.norm = nn.LayerNorm(embed_dim)
        self.dropout = nn.Dropout(dropout)

    def forward(self, department_ids, category_ids):
        from .ops import category_hierarchy_forward
        return category_hierarchy_forward(self, department_ids, category_ids)


class _NCFTrainFunction(torch.autograd.Function):
    """Forward + backward of AdvancedNCF.forward in training mode.  The last input is the
    model's grad anchor (a 0-element tensor that requires grad), which connects the output to
    autograd at the cost of one input instead of every parameter's; the gradients are written
    by the kernels directly (dense: views of the engine's flat gradient buffer, assigned as
    .grad; tables: compact rows, applied by the fused Adam or materialised on demand).

    With a deferred table schedule attached (optim.py binding / FusedTrainStep), the forward
    deduplicates the batch ids and catches exactly those rows up first (deferred.prepare)."""

    @staticmethod
    def forward(ctx, engine, uid, iid, M, drop_p, seed, anchor):
        d = engine.deferred
        # a step left unapplied (e.g. accumulation) keeps its rows' gradients in the
        # workspace this forward reuses: make them dense table .grad before they are overwritten
        _settle_pending(engine, uid.device)
        tp = engine.tapes
        w = tp.forward(uid, iid, M, drop_p, seed) if tp is not None else None
        if w is None:
            w = engine.forward(uid, iid, M, True, drop_p, seed,
                               prepare=d.prepare if d is not None else None)
        ctx.engine, ctx.w, ctx.drop_p, ctx.seed = engine, w, drop_p, seed
        ctx.save_for_backward(uid, iid)
        return w.prob.view(-1, 1).clone()

    @staticmethod
    def backward(ctx, grad_out):
        uid, iid = ctx.saved_tensors
        eng = ctx.engine
        views = eng.grad_views()
        prev = [(p, p.grad.clone()) for p, _ in views if p.grad is not None and p.requires_grad]
        _settle_pending(eng, grad_out.device)
        gp = grad_out.reshape(-1).to(torch.float32).contiguous()
        tp = eng.tapes
        if tp is None or not tp.backward(ctx.w, uid, iid, gp, ctx.drop_p, ctx.seed):
            eng.backward(ctx.w, uid, iid, gp, None, ctx.drop_p, ctx.seed)
        for p, v in views:
            if p.requires_grad:
                p.grad = v
        for p, g in prev:  # gradient accumulation across backward() calls
            p.grad.add_(g)
        eng.grad_version = eng.flat_grad._version
        return (None,) * 7


def _settle_pending(eng, device):
    """Compact table gradients of a backward whose optimizer step has not run yet: kept (as
    dense table .grad, summed with the next ones) when the dense gradients of that backward
    are still there untouched — gradient accumulation — and dropped when they were cleared
    in between (zero_grad: set to None, or zeroed in place, which bumps their version)."""
    if eng.pending is None:
        return
    views = eng.grad_views()
    kept = any(p.grad is v for p, v in views) and \
        getattr(eng, "grad_version", None) == eng.flat_grad._version
    if kept:
        eng.materialize_table_grads(accumulate=True)
    else:
        eng.release_pending(_lib.stream_ptr(device))


class AdvancedNCF(nn.Module):
    def __init__(self,
                 num_users: int,
                 num_products: int,
                 num_departments: int,
                 num_categories: int,
                 mf_embedding_dim: int = 64,
                 mlp_embedding_dim: int = 64,
                 temporal_dim: int = 32,
                 mlp_hidden_dims: List[int] = [256, 128, 64],
                 num_heads: int = 4,
                 dropout: float = 0.2,
                 negative_samples: int = 4):
        super().__init__()
        self.num_users = num_users
        self.num_products = num_products
        self.num_departments = num_departments
        self.num_categories = num_categories
        self.mf_embedding_dim = mf_embedding_dim
        self.mlp_embedding_dim = mlp_embedding_dim
        self.mf_norm = nn.LayerNorm(mf_embedding_dim)
        self.mlp_norm = nn.LayerNorm(mlp_embedding_dim)
        self.temporal_dim = temporal_dim
        self.mlp_hidden_dims = list(mlp_hidden_dims)
        self.num_heads = num_heads
        self.dropout = dropout
        self.negative_samples = negative_samples

        def ebc(dim):
            return EmbeddingBagCollection(tables=[
                EmbeddingBagConfig(name="user_id", embedding_dim=dim, num_embeddings=num_users,
                                   feature_names=["user_id"], pooling=PoolingType.SUM),
                EmbeddingBagConfig(name="product_id", embedding_dim=dim,
                                   num_embeddings=num_products, feature_names=["product_id"],
                                   pooling=PoolingType.SUM)])

        self.mf_embedding_collection = ebc(mf_embedding_dim)            # :153-170
        self.mlp_embedding_collection = ebc(mlp_embedding_dim)          # :173-190
        self.category_hierarchy = CategoryHierarchy(num_departments, num_categories,
                                                    mlp_embedding_dim, dropout)   # :193-198
        self.temporal_encoding = TemporalEncoding(temporal_dim)         # :201
        self.user_product_attention = MultiHeadAttention(mlp_embedding_dim, num_heads, dropout)
        self.sequence_attention = MultiHeadAttention(mlp_embedding_dim, num_heads, dropout)
        combined_dim = mlp_embedding_dim + temporal_dim                  # :217-220
        self.feature_combination = nn.Sequential(
            nn.Linear(combined_dim, mlp_hidden_dims[0]), nn.ReLU(),
            nn.LayerNorm(mlp_hidden_dims[0]), nn.Dropout(dropout))
        layers, cur = [], combined_dim                                   # :230-242
        for h in mlp_hidden_dims:
            layers += [nn.Linear(cur, h), nn.ReLU(), nn.LayerNorm(h), nn.Dropout(dropout)]
            cur = h
        self.mlp = nn.Sequential(*layers)
        self.mf_output = nn.Linear(mf_embedding_dim, 1)                  # :245
        self.mlp_output = nn.Linear(mlp_hidden_dims[-1], 1)              # :246
        self.final = nn.Sequential(nn.Linear(2, 1), nn.Sigmoid())        # :249-252
        self.mf_norm = nn.LayerNorm(mf_embedding_dim)                    # :255-256 (re-created;
        self.mlp_norm = nn.LayerNorm(mlp_embedding_dim)                  #  keeps key order)
        object.__setattr__(self, "_engine", NCFEngine(self))
        # autograd anchor of the training forward (not a parameter or buffer: no state_dict key)
        object.__setattr__(self, "_anchor", torch.zeros(0, requires_grad=True))
        self._engine.flatten()
        eref = weakref.ref(self._engine)

        def sync():
            e = eref()
            if e is not None:
                e.sync_tables()
        self.mf_embedding_collection.set_sync(sync)
        self.mlp_embedding_collection.set_sync(sync)
        _optim.register(self)

    # keep the dense flat layout valid across .to()/.cuda()/.float()
    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        self._engine.flatten()
        return out

    @property
    def engine(self) -> NCFEngine:
        return self._engine

    def state_dict(self, *args, **kwargs):
        # a deferred optimizer may hold untouched table rows behind: materialise them first
        self._engine.sync_tables()
        return super().state_dict(*args, **kwargs)

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        # rows a deferred optimizer still owes zero-gradient steps must settle BEFORE they are
        # overwritten: otherwise the owed steps (decay + old moments) would later be replayed
        # onto the loaded values.  After the sweep every row is current, so the loaded rows
        # simply continue from the optimizer's current step (as with torch's dense Adam).
        self._engine.sync_tables()
        out = super().load_state_dict(state_dict, strict=strict, assign=assign)
        self._engine.updates += 1
        if self._engine.deferred is not None:     # bf16 tables take the loaded values
            self._engine.deferred.reload_params()
        if assign:
            self._engine.flatten()
        return out

    # ---------------------------------------------------------------- forward (:258-381)
    def forward(self, features: KeyedJaggedTensor) -> torch.Tensor:
        total_samples = features.values().size(0) // 2                  # :274
        M = 1 + self.negative_samples if self.training else 1           # :275
        ids = features.single_id_split()
        uid, iid = ids["user_id"], ids["product_id"]
        if uid.numel() != total_samples or iid.numel() != total_samples:
            raise ValueError(f"embedding shape mismatch: got {uid.numel()}/{iid.numel()}, "
                             f"expected {total_samples}")                 # :298-302
        eng = self._engine
        train = self.training and torch.is_grad_enabled()
        drop_p = float(self.dropout) if self.training else 0.0
        # with a device step clock attached (the fused Adam bound to this model) the kernels
        # draw their dropout stream from the clock's per-step seed, as FusedTrainStep does
        seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if drop_p > 0 and eng.clock is None else 0
        if train:
            dev = eng.flat.device if eng.flat is not None else uid.device
            uid = uid.to(device=dev, dtype=torch.int64).contiguous()   # (the engine's own
            iid = iid.to(device=dev, dtype=torch.int64).contiguous()   #  conversion, once)
            out = _NCFTrainFunction.apply(eng, uid, iid, M, drop_p, seed, self._anchor)
        else:
            w = eng.forward(uid, iid, M, False, drop_p, seed)
            out = w.prob.view(-1, 1).clone()
        v = getattr(self, "validate_ids", True)
        if v:
            ws = eng.ws[(uid.numel(), M, train)]
            if train and v != "sync":
                eng.check_ids_async(ws)      # no host sync inside the training loop
            else:
                eng.check_ids(ws)
        if not hasattr(self, "_first_forward_done"):                    # :365-372
            log.info("First forward pass: output %s", tuple(out.shape))
            self._first_forward_done = True
        return out

    def forward_simple(self, user_ids, product_ids, hour=None):
        """(:409-485) With hour=None this is the eval forward with M=1 per pair; with hour the
        reference's temporal variant, including its fresh random projection per call."""
        if hour is not None:
            from .ops import forward_simple_hour
            if (self.training and torch.is_grad_enabled()
                    and any(p.requires_grad for p in self.parameters())):
                # (its forward runs in training mode, dropout included, under torch.no_grad())
                raise NotImplementedError("forward_simple(hour=...) has no backward on the "
                                          "accelerated path; call it under torch.no_grad()")
            return forward_simple_hour(self, user_ids, product_ids, hour)
        eng = self._engine
        if self.training and torch.is_grad_enabled():
            # training mode (the reference's nn.Dropout layers active): the training forward with
            # one item per group — the attention over a single key — through the same autograd
            # function as forward(), so loss.backward() reaches every parameter; the dropout
            # masks come from this package's stream (as in forward())
            drop_p = float(self.dropout)
            seed = (int(torch.randint(0, 2 ** 62, (1,)).item())
                    if drop_p > 0 and eng.clock is None else 0)
            dev = eng.flat.device if eng.flat is not None else user_ids.device
            uid = user_ids.reshape(-1).to(device=dev, dtype=torch.int64).contiguous()
            iid = product_ids.reshape(-1).to(device=dev, dtype=torch.int64).contiguous()
            if uid.numel() != iid.numel():
                raise ValueError("forward_simple: user_ids and product_ids differ in length")
            out = _NCFTrainFunction.apply(eng, uid, iid, 1, drop_p, seed, self._anchor)
            v = getattr(self, "validate_ids", True)
            if v:
                ws = eng.ws[(uid.numel(), 1, True)]
                if v != "sync":
                    eng.check_ids_async(ws)
                else:
                    eng.check_ids(ws)
            return out.view(-1)
        w = eng.forward(user_ids, product_ids, 1, False, 0.0, 0)
        eng.check_ids(w)
        return w.prob.clone()

    def get_user_embeddings(self, user_features: Dict) -> Dict[str, torch.Tensor]:
        """(:383-391)"""
        self._engine.sync_tables()
        ids = user_features["user_features"].single_id_split()["user_id"]
        return {"mf": gather_rows(self.mf_embedding_collection.embedding_bags["user_id"].weight,
                                  ids, self.mf_norm.weight, self.mf_norm.bias, LN_EPS),
                "mlp": gather_rows(self.mlp_embedding_collection.embedding_bags["user_id"].weight,
                                   ids, self.mlp_norm.weight, self.mlp_norm.bias, LN_EPS)}

    def get_product_embeddings(self, product_features: Dict) -> Dict[str, torch.Tensor]:
        """(:393-407)"""
        self._engine.sync_tables()
        ids = product_features["product_features"].single_id_split()["product_id"]
        cat = self.category_hierarchy(product_features["category_features"]["department_ids"],
                                      product_features["category_features"]["category_ids"])
        return {"mf": gather_rows(self.mf_embedding_collection.embedding_bags["product_id"].weight,
                                  ids, self.mf_norm.weight, self.mf_norm.bias, LN_EPS),
                "mlp": gather_rows(self.mlp_embedding_collection.embedding_bags["product_id"].weight,
                                   ids, self.mlp_norm.weight, self.mlp_norm.bias, LN_EPS),
                "category": cat}
