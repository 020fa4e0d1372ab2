"""Item-embedding export for the ANN index.

The reference's ``generate_embeddings.py`` walks the exported product rows, maps each
``product_id`` to a table row (``int(product_id.lstrip('P'), 16) % num_products``, :106),
calls ``model.get_product_embeddings`` one product at a time, takes the ``"mlp"`` vector
(LayerNorm'd MLP item row), L2-normalises it and writes one JSON line
``{"id": product_id, "embedding": [...]}`` per distinct product (:193-221); the JSONL feeds
a Vertex AI Tree-AH index with cosine distance (setup_tree_ah_endpoint.py:25-32).

Here the vectors of all products come from one launch of the gather + LayerNorm kernel with
the L2 normalisation fused (``ncf_embedding_export``); the JSON lines are written on the host in
the reference's format.  GPU only for the vectors (no CPU fallback).
"""
import json
from typing import IO, Iterable, List, Mapping, Sequence, Tuple, Union

import torch

from . import _lib
from ._lib import ptr
from .engine import LN_EPS


def product_index(product_id: str, num_products: int) -> int:
    """generate_embeddings.py:106 — hex product code (optional 'P' prefix) modulo the table."""
    return int(product_id.lstrip("P"), 16) % num_products


def product_embeddings(model, product_idx: torch.Tensor, normalize: bool = True,
                       table: str = "mlp") -> torch.Tensor:
    """``get_product_embeddings(...)[table]`` rows for ``product_idx`` (LayerNorm'd, then
    L2-normalised when ``normalize``): ``[n, D]`` fp32 on the model's device."""
    model._engine.sync_tables()
    dev = model.mlp_norm.weight.device
    if dev.type != "cuda":
        raise RuntimeError("ncf_amd export runs on the MI355X only (no CPU fallback)")
    coll, ln = ((model.mlp_embedding_collection, model.mlp_norm) if table == "mlp" else
                (model.mf_embedding_collection, model.mf_norm))
    w = coll.embedding_bags["product_id"].weight
    ids = product_idx.to(device=dev, dtype=torch.int64).contiguous()
    out = torch.empty(ids.numel(), w.shape[1], device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.call("ncf_embedding_export", ptr(ids), ids.numel(), ptr(w), w.shape[0], w.shape[1],
              ptr(ln.weight), ptr(ln.bias), LN_EPS, 1 if normalize else 0, ptr(out), ptr(err),
              _lib.stream_ptr(dev))
    if int(err.item()):
        raise IndexError("product index out of range of the embedding table")
    return out


def write_embeddings_jsonl(out: Union[str, IO[str]], ids: Sequence[str],
                           embeddings: torch.Tensor) -> int:
    """One ``{"id": ..., "embedding": [...]}`` JSON line per row (generate_embeddings.py:213-218);
    returns the number of lines written."""
    vecs = embeddings.detach().to("cpu", torch.float32).numpy()
    if len(ids) != vecs.shape[0]:
        raise ValueError("ids and embeddings differ in length")
    fh = open(out, "w") if isinstance(out, str) else out
    try:
        for pid, v in zip(ids, vecs):
            fh.write(json.dumps({"id": str(pid), "embedding": v.tolist()}) + "\n")
    finally:
        if isinstance(out, str):
            fh.close()
    return len(ids)


def distinct_products(rows: Iterable[Mapping], num_products: int) -> Tuple[List[str], List[int]]:
    """The reference's row filter (generate_embeddings.py:193-203): skip rows without a
    product_id and repeats; returns (product ids, table rows) in first-seen order."""
    seen, pids, idx = set(), [], []
    for row in rows:
        pid = row.get("product_id")
        if not pid or pid in seen:
            continue
        seen.add(pid)
        pids.append(str(pid))
        idx.append(product_index(str(pid), num_products))
    return pids, idx


def export_product_embeddings(model, rows: Iterable[Mapping], out: Union[str, IO[str]],
                              batch: int = 1 << 20) -> int:
    """The export loop of generate_embeddings.py (:193-221) minus the GCS transfer: distinct
    products of ``rows`` -> L2-normalised "mlp" vectors -> JSONL at ``out``."""
    pids, idx = distinct_products(rows, model.num_products)
    fh = open(out, "w") if isinstance(out, str) else out
    try:
        n = 0
        for s in range(0, len(pids), batch):
            e = product_embeddings(model, torch.tensor(idx[s:s + batch], dtype=torch.int64))
            n += write_embeddings_jsonl(fh, pids[s:s + batch], e)
    finally:
        if isinstance(out, str):
            fh.close()
    return n
