"""torchrec-compatible sparse input types and the EmbeddingBagCollection used by AdvancedNCF.

The reference imports ``EmbeddingBagCollection, EmbeddingBagConfig, PoolingType`` from torchrec
and ``KeyedJaggedTensor`` from ``torchrec.sparse.jagged_tensor`` (src/model/architecture.py:5-12,
src/model/data_prep.py:5, src/inference/*).  torchrec (0.8.0, Dockerfile:23-25) is not part of
this framework: these classes provide the surface those call sites use —
``KeyedJaggedTensor(keys, values, lengths=None, offsets=None)``, ``.from_lengths_sync``,
``keys() / values() / lengths() / offsets() / to() / to_dict() / __getitem__`` — and an EBC whose
parameters are named ``embedding_bags.<table>.weight`` (the reference state_dict keys).

The EBC forward is the HIP row gather (single-id SUM bags == one row per bag, which is how every
reference call site builds its KJTs: lengths == 1, data_prep.py:273-283, architecture.py:418-422).
"""
import enum
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch
import torch.nn as nn

from . import _lib


class PoolingType(enum.Enum):
    SUM = "SUM"
    MEAN = "MEAN"
    NONE = "NONE"


@dataclass
class EmbeddingBagConfig:
    num_embeddings: int
    embedding_dim: int
    name: str = ""
    feature_names: List[str] = field(default_factory=list)
    pooling: PoolingType = PoolingType.SUM
    weight_init_max: Optional[float] = None
    weight_init_min: Optional[float] = None


class JaggedTensor:
    def __init__(self, values: torch.Tensor, lengths: torch.Tensor):
        self._values = values
        self._lengths = lengths

    def values(self):
        return self._values

    def lengths(self):
        return self._lengths

    def offsets(self):
        z = torch.zeros(1, dtype=self._lengths.dtype, device=self._lengths.device)
        return torch.cat([z, torch.cumsum(self._lengths, 0)])


class KeyedJaggedTensor:
    """Keyed jagged ids: ``values`` = concatenation over keys; ``lengths`` has
    ``len(keys) * stride`` entries (per key, one length per bag)."""

    def __init__(self, keys: List[str], values: torch.Tensor, lengths: Optional[torch.Tensor] = None,
                 offsets: Optional[torch.Tensor] = None, weights=None, stride: Optional[int] = None,
                 **kwargs):
        self._keys = list(keys)
        self._values = values
        if lengths is None:
            if offsets is None:
                raise ValueError("KeyedJaggedTensor needs lengths or offsets")
            lengths = offsets[1:] - offsets[:-1]
        self._lengths = lengths
        self._weights = weights
        if stride is None:
            stride = lengths.numel() // max(1, len(self._keys))
        self._stride = stride

    @staticmethod
    def from_lengths_sync(keys, values, lengths, weights=None, stride=None):
        return KeyedJaggedTensor(keys, values, lengths=lengths, weights=weights, stride=stride)

    @staticmethod
    def from_offsets_sync(keys, values, offsets, weights=None, stride=None):
        return KeyedJaggedTensor(keys, values, offsets=offsets, weights=weights, stride=stride)

    def keys(self) -> List[str]:
        return self._keys

    def values(self) -> torch.Tensor:
        return self._values

    def lengths(self) -> torch.Tensor:
        return self._lengths

    def offsets(self) -> torch.Tensor:
        z = torch.zeros(1, dtype=self._lengths.dtype, device=self._lengths.device)
        return torch.cat([z, torch.cumsum(self._lengths, 0)])

    def weights_or_none(self):
        return self._weights

    def stride(self) -> int:
        return self._stride

    @property
    def device(self):
        return self._values.device

    def to(self, device, non_blocking: bool = False) -> "KeyedJaggedTensor":
        return KeyedJaggedTensor(self._keys, self._values.to(device, non_blocking=non_blocking),
                                 lengths=self._lengths.to(device, non_blocking=non_blocking),
                                 stride=self._stride)

    def pin_memory(self):
        return KeyedJaggedTensor(self._keys, self._values.pin_memory(),
                                 lengths=self._lengths.pin_memory(), stride=self._stride)

    def single_id_split(self) -> Dict[str, torch.Tensor]:
        """{key: ids} for the single-id-bag layout (every length == 1): key k owns
        values[k*stride:(k+1)*stride].  Raises NotImplementedError for pooled bags."""
        n = len(self._keys) * self._stride
        if self._values.numel() != n or self._lengths.numel() != n:
            raise NotImplementedError("AdvancedNCF path supports single-id bags (lengths == 1) only")
        if self._lengths.device.type == "cpu" and n and not bool((self._lengths == 1).all()):
            raise NotImplementedError("AdvancedNCF path supports single-id bags (lengths == 1) only")
        s = self._stride
        return {k: self._values[i * s:(i + 1) * s] for i, k in enumerate(self._keys)}

    def to_dict(self) -> Dict[str, JaggedTensor]:
        out, pos = {}, 0
        cum = torch.cumsum(self._lengths, 0).tolist() if self._lengths.numel() else []
        for i, k in enumerate(self._keys):
            a = i * self._stride
            b = (i + 1) * self._stride
            end = cum[b - 1] if b > 0 and cum else 0
            out[k] = JaggedTensor(self._values[pos:end], self._lengths[a:b])
            pos = end
        return out

    def __getitem__(self, key: str) -> JaggedTensor:
        return self.to_dict()[key]

    def __repr__(self):
        return (f"KeyedJaggedTensor(keys={self._keys}, values={tuple(self._values.shape)}, "
                f"stride={self._stride})")


class _Bag(nn.Module):
    """Holds one table; the parameter is named ``weight`` like nn.EmbeddingBag.

    A deferred dense-exact optimizer (deferred.py) may hold rows of the table behind the step
    count; every read of the table through this module — ``bag.weight``, ``state_dict()`` of
    the bag or of any module above it, the collection's forward — first brings them current
    (``_sync``, installed by the owning AdvancedNCF).  The kernels use ``raw_weight()``."""

    def __init__(self, num_embeddings: int, embedding_dim: int):
        super().__init__()
        self.num_embeddings = num_embeddings
        self.embedding_dim = embedding_dim
        self._sync = None
        self.weight = nn.Parameter(torch.empty(num_embeddings, embedding_dim))
        self.register_state_dict_pre_hook(_bag_state_dict_pre)

    @property
    def weight(self):
        p = self.__dict__["_parameters"].get("weight")
        if p is None:
            raise AttributeError("weight")
        s = self.__dict__.get("_sync")
        if s is not None:
            s()
        return p

    def raw_weight(self) -> nn.Parameter:
        """The parameter itself, without bringing lagging rows current (kernel plumbing)."""
        return self._parameters["weight"]


def _bag_state_dict_pre(module, prefix, keep_vars):
    s = module.__dict__.get("_sync")
    if s is not None:
        s()


class EmbeddingBagCollection(nn.Module):
    """Drop-in for torchrec.EmbeddingBagCollection on the AdvancedNCF path."""

    def __init__(self, tables: List[EmbeddingBagConfig], device=None, is_weighted: bool = False):
        super().__init__()
        self._embedding_bag_configs = list(tables)
        self.embedding_bags = nn.ModuleDict()
        for t in self._embedding_bag_configs:
            if t.pooling not in (PoolingType.SUM, PoolingType.MEAN):
                raise ValueError("EmbeddingBagCollection supports SUM/MEAN pooling")
            bag = _Bag(t.num_embeddings, t.embedding_dim)
            # torchrec default init: U(-sqrt(1/rows), sqrt(1/rows))
            bound = (1.0 / max(1, t.num_embeddings)) ** 0.5
            lo = -bound if t.weight_init_min is None else t.weight_init_min
            hi = bound if t.weight_init_max is None else t.weight_init_max
            with torch.no_grad():
                bag.weight.uniform_(lo, hi)
            self.embedding_bags[t.name] = bag
        if device is not None:
            self.to(device)

    def embedding_bag_configs(self):
        return self._embedding_bag_configs

    def table_for(self, feature: str) -> _Bag:
        for t in self._embedding_bag_configs:
            if feature in t.feature_names:
                return self.embedding_bags[t.name]
        raise KeyError(feature)

    def forward(self, features: KeyedJaggedTensor) -> Dict[str, torch.Tensor]:
        ids = features.single_id_split()
        out = {}
        for t in self._embedding_bag_configs:
            bag = self.embedding_bags[t.name]
            for f in t.feature_names:
                if f in ids:
                    out[f] = gather_rows(bag.weight, ids[f])   # (.weight: rows current)
        return out

    def set_sync(self, fn):
        """Install the callable that brings lagging table rows current before a read."""
        for bag in self.embedding_bags.values():
            bag._sync = fn


def gather_rows(table: torch.Tensor, ids: torch.Tensor, gamma=None, beta=None, eps=1e-5) -> torch.Tensor:
    """HIP row gather (+ optional LayerNorm); rows of ``table`` at int64 ``ids``."""
    if table.device.type != "cuda":
        raise RuntimeError("ncf_amd: the AdvancedNCF path runs on the GPU only (no CPU fallback); "
                           "move the model to cuda")
    ids = ids.to(device=table.device, dtype=torch.int64).contiguous()
    table = table.detach()
    out = torch.empty(ids.numel(), table.shape[1], device=table.device, dtype=torch.float32)
    err = torch.zeros(1, dtype=torch.int32, device=table.device)
    _lib.call("ncf_gather_rows", _lib.ptr(ids), ids.numel(), _lib.ptr(table), table.shape[0],
              table.shape[1], _lib.ptr(gamma), _lib.ptr(beta), eps, _lib.ptr(out), _lib.ptr(err),
              _lib.stream_ptr(table.device))
    if int(err.item()):
        raise IndexError("embedding id out of range")
    return out
