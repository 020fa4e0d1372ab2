"""ncf_amd — MI355X-native (gfx950 / CDNA4) AdvancedNCF training + scoring hot path.

Drop-in for the reference's ``src.model.architecture`` surface (AdvancedNCF, MultiHeadAttention,
TemporalEncoding, CategoryHierarchy) and the torchrec types it consumes (KeyedJaggedTensor,
EmbeddingBagCollection, EmbeddingBagConfig, PoolingType).  Compute runs in hand-written HIP
kernels (libncf_hip.so, C-ABI in include/ncf_hip.h); there is no CPU fallback.

This directory's name (``neural-collaborative-filtering-demo_amd``) is not a Python identifier;
``_ncf_pkg.load()`` at the repo root registers it as the importable package ``ncf_amd``.
"""
from ._lib import LIB_PATH, NCFLibraryError, load as load_library  # noqa: F401
from .sparse import (EmbeddingBagCollection, EmbeddingBagConfig, JaggedTensor,  # noqa: F401
                     KeyedJaggedTensor, PoolingType)
from .architecture import (AdvancedNCF, CategoryHierarchy, MultiHeadAttention,  # noqa: F401
                           TemporalEncoding)

__version__ = "1.0.0"
