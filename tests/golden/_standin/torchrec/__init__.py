"""Offline torchrec stand-in used ONLY by tests/golden/make_goldens.py to import the
reference's src/model/architecture.py in the survey container (torchrec==0.8.0 is not
installed and cannot be fetched offline).  It restates the tiny slice of torchrec the
reference touches: EmbeddingBagConfig/PoolingType/EmbeddingBagCollection (parameter
names ``embedding_bags.<table>.weight``) and KeyedJaggedTensor.  Single-id SUM bags are
a plain row gather; that identity is pinned by the demo checkpoint reproducing the
reference's committed predictions.csv.  Never shipped, never imported by the product.
"""
import enum
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.nn as nn

from .sparse.jagged_tensor import KeyedJaggedTensor  # noqa: F401


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


class EmbeddingBagCollection(nn.Module):
    def __init__(self, tables, device=None, is_weighted=False):
        super().__init__()
        self._tables = list(tables)
        self.embedding_bags = nn.ModuleDict()
        for t in self._tables:
            mode = {"SUM": "sum", "MEAN": "mean"}[t.pooling.value]
            bag = nn.EmbeddingBag(t.num_embeddings, t.embedding_dim, mode=mode,
                                  include_last_offset=True)
            bound = (1.0 / t.num_embeddings) ** 0.5
            lo = -bound if t.weight_init_min is None else t.weight_init_min
            hi = bound if t.weight_init_max is None else t.weight_init_max
            with torch.no_grad():
                bag.weight.uniform_(lo, hi)
            self.embedding_bags[t.name] = bag

    def forward(self, features):
        d = features.to_dict()
        out = {}
        for t in self._tables:
            for f in t.feature_names:
                jt = d[f]
                out[f] = self.embedding_bags[t.name](jt.values(), jt.offsets())
        return out
