"""Device-side training batches: inverse-popularity negatives + the KJT rows.

The reference builds every training row on the host: ``SheetzDataset.__getitem__`` draws each
negative with ``np.random.choice(num_products, p=product_weights)`` (O(I) per draw) and rejects
the user's positives (src/model/data_prep.py:134-161, 181-228), then
``collate_recommender_batch`` loops over every id in Python to build the
``KeyedJaggedTensor`` (:230-313).  ``DeviceNegativeSampler`` keeps the interaction list, an
alias table of the same weights and the users' histories in HBM, and ``batch`` produces the
collated ``(KeyedJaggedTensor, targets [N, 1])`` for a set of interaction indices in one HIP
launch (csrc/sampler.hip), ready for ``model(kjt)`` / ``FusedTrainStep``.

    sampler = DeviceNegativeSampler(users, products, num_users, num_products, negative_samples=4)
    for kjt, targets in sampler.epoch(batch_size=256, seed=epoch):
        ...

Same weights (1 / max(count, 1), normalised; data_prep.py:95-102), same rejection rule
(positive + user history, 10 attempts, then uniform over the non-history items, data_prep.py
:141-161), same row layout and targets; the draw stream is the device counter hash (the numpy
draw order is excluded from parity).  GPU only (no CPU fallback); the alias table is
built on the host once (``ncf_alias_build``).
"""
from typing import Iterator, Optional, Tuple

import numpy as np
import torch

from . import _lib
from ._lib import ptr
from .sparse import KeyedJaggedTensor


def inverse_popularity_weights(products: torch.Tensor, num_products: int) -> np.ndarray:
    """data_prep.py:95-102: counts per product, clamped to >= 1, inverted, normalised (f64)."""
    counts = torch.bincount(products.to(torch.int64).cpu(), minlength=num_products)[:num_products]
    w = 1.0 / np.maximum(counts.numpy().astype(np.float64), 1.0)
    return w / w.sum()


def alias_table(weights: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Walker/Vose alias table (host, O(n)) of ``weights``: (prob f32 [n], alias i32 [n])."""
    w = np.ascontiguousarray(weights, dtype=np.float64)
    prob = np.empty(w.size, dtype=np.float32)
    alias = np.empty(w.size, dtype=np.int32)
    _lib.call("ncf_alias_build", w.ctypes.data, w.size, prob.ctypes.data, alias.ctypes.data)
    return prob, alias


class ConsistentBatchSampler:
    """The reference's training batch sampler (src/model/data_prep.py:397-443), same
    constructor and iteration: ``num_batches = ceil(size / batch_size)`` index lists over
    ``range(dataset_size)`` (shuffled in place by ``np.random.shuffle`` when ``shuffle``); a short
    last batch is extended with ``batch[:batch_size - len(batch)]``, i.e. with repeats of its own
    first indices, so it stays short when it holds fewer than half a batch (data_prep.py:436-438).
    For ``torch.utils.data.DataLoader(batch_sampler=...)`` on the host; on the device
    ``DeviceNegativeSampler.epoch`` applies the same padding rule."""

    def __init__(self, dataset_size: int, batch_size: int, shuffle: bool = True):
        self.dataset_size = dataset_size
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.num_batches = (dataset_size + batch_size - 1) // batch_size
        self.last_batch_size = dataset_size % batch_size or batch_size

    def __iter__(self):
        indices = list(range(self.dataset_size))
        if self.shuffle:
            np.random.shuffle(indices)
        for b in range(self.num_batches):
            batch = indices[b * self.batch_size:(b + 1) * self.batch_size]
            short = self.batch_size - len(batch)
            if short > 0:
                batch.extend(batch[:short])
            yield batch

    def __len__(self) -> int:
        return self.num_batches


class DeviceNegativeSampler:
    """Interaction list + negative sampler + collate, resident on the GPU."""

    def __init__(self, users: torch.Tensor, products: torch.Tensor, num_users: int,
                 num_products: int, negative_samples: int = 4, mode: str = "train",
                 device=None, max_attempts: int = 10):
        if mode not in ("train", "val"):
            raise ValueError("mode must be 'train' or 'val'")
        device = torch.device(device or "cuda")
        if device.type != "cuda":
            raise RuntimeError("DeviceNegativeSampler runs on the MI355X only (no CPU fallback)")
        users = torch.as_tensor(users, dtype=torch.int64).reshape(-1)
        products = torch.as_tensor(products, dtype=torch.int64).reshape(-1)
        if users.numel() != products.numel():
            raise ValueError("users and products must have the same length")
        if users.numel() and (int(users.min()) < 0 or int(users.max()) >= num_users or
                              int(products.min()) < 0 or int(products.max()) >= num_products):
            raise IndexError("interaction ids out of range")
        self.mode = mode
        self.negative_samples = negative_samples if mode == "train" else 0
        self.num_users, self.num_products = num_users, num_products
        self.max_attempts = max_attempts
        self.device = device
        self.users = users.to(device)
        self.products = products.to(device)
        self.weights = inverse_popularity_weights(products, num_products)
        prob, alias = alias_table(self.weights)
        self.alias_prob = torch.from_numpy(prob).to(device)
        self.alias_idx = torch.from_numpy(alias).to(device)
        # user -> sorted unique positive products (data_prep.py:163-176), CSR on the device
        key = torch.unique(users * num_products + products)
        hu, hi = key // num_products, key % num_products
        self.hist_offsets = torch.zeros(num_users + 1, dtype=torch.int64)
        self.hist_offsets[1:] = torch.cumsum(torch.bincount(hu, minlength=num_users), 0)
        self.hist_offsets = self.hist_offsets.to(device)
        self.hist_items = hi.to(torch.int32).to(device)
        self._err = torch.zeros(1, dtype=torch.int32, device=device)

    def __len__(self) -> int:
        return self.users.numel()

    def batch(self, indices: torch.Tensor, seed: int) -> Tuple[KeyedJaggedTensor, torch.Tensor]:
        """Collated batch for interaction ``indices``: KJT values ``[users || items]`` (each id
        its own bag) and targets ``[N, 1]``, N = len(indices) * (1 + negative_samples)."""
        idx = torch.as_tensor(indices, dtype=torch.int64).to(self.device).reshape(-1)
        B, M = idx.numel(), 1 + self.negative_samples
        u = self.users.index_select(0, idx)
        p = self.products.index_select(0, idx)
        out_u = torch.empty(B * M, dtype=torch.int64, device=self.device)
        out_i = torch.empty(B * M, dtype=torch.int64, device=self.device)
        tgt = torch.empty(B * M, dtype=torch.float32, device=self.device)
        _lib.call("ncf_sample_negatives", ptr(u), ptr(p), B, self.negative_samples,
                  ptr(self.alias_prob), ptr(self.alias_idx), self.num_products,
                  ptr(self.hist_offsets), ptr(self.hist_items), self.num_users,
                  seed & (2 ** 64 - 1), self.max_attempts, ptr(out_u), ptr(out_i), ptr(tgt),
                  ptr(self._err), _lib.stream_ptr(self.device))
        kjt = KeyedJaggedTensor.from_lengths_sync(
            keys=["user_id", "product_id"], values=torch.cat([out_u, out_i]),
            lengths=torch.ones(2 * B * M, dtype=torch.int64, device=self.device))
        return kjt, tgt.unsqueeze(1)

    def epoch(self, batch_size: int, seed: int = 0, shuffle: bool = True,
              drop_last: bool = False, pad_last: Optional[bool] = None
              ) -> Iterator[Tuple[KeyedJaggedTensor, torch.Tensor]]:
        """One pass over the interactions in batches (the DataLoader + collate loop of
        trainer.py:134-140, 253-258), order and negatives a function of ``seed``.

        ``pad_last`` (default: train mode) is the reference's training loader, whose
        ``ConsistentBatchSampler`` (data_prep.py:397-443, used at trainer.py:127-140) pads a short
        last batch with the first indices of that same batch (at most doubling it); without it
        the last batch is short (the validation loader, trainer.py:142-148)."""
        n = len(self)
        if pad_last is None:
            pad_last = self.mode == "train"
        if shuffle:
            g = torch.Generator(device=self.device).manual_seed(seed)
            order = torch.randperm(n, generator=g, device=self.device)
        else:
            order = torch.arange(n, device=self.device)
        for b, s in enumerate(range(0, n, batch_size)):
            chunk = order[s:s + batch_size]
            if drop_last and chunk.numel() < batch_size:
                break
            if pad_last and chunk.numel() < batch_size:
                chunk = torch.cat([chunk, chunk[:batch_size - chunk.numel()]])
            yield self.batch(chunk, (seed * 1_000_003 + b) & (2 ** 63 - 1))

    def check(self):
        """Raise if any batch so far held an out-of-range id (one host sync)."""
        if int(self._err.item()):
            raise IndexError("DeviceNegativeSampler: interaction id out of range")
