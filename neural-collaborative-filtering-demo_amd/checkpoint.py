"""Checkpoint I/O compatible with the reference's artifacts.

* Trainer checkpoints (src/model/trainer.py:548-609): ``{epoch, model_state_dict,
  optimizer_state_dict, metrics, config, model_config, [scheduler_state_dict]}`` written with
  ``torch.save``; ``load_checkpoint`` restores model + optimizer and returns ``epoch + 1``.
  The optimizer may be a ``torch.optim.Adam`` (the reference trainer; state is kept in torch's
  format by ncf_amd.optim) or a ``FusedTrainStep`` (its moments are exported to / imported from
  the same torch Adam ``state_dict`` format, so either side can resume the other's files).
* Bare ``state_dict`` artifacts (src/train.py:86-91): ``save_model`` / ``load_model``.
* Sharded -> single:
  - ``load_unzipped_archive``: a ``torch.save`` archive that was unzipped into a directory
    (``data.pkl``, ``data/<key>``, ``version``, ...) — what consolidate_shards.py
    (src/inference/demo/consolidate_shards.py:72-116) rebuilds by matching raw tensor sizes —
    is re-zipped in memory and read by the archive's own record of keys, shapes and strides;
  - ``consolidate_row_shards`` / ``shard_state_dict``: the row-sharded tables of the
    multi-GPU step (ncf_amd.distributed: rank r owns rows ``id % W == r``) to / from one
    full ``state_dict``.
Every load goes through ``torch.load(..., weights_only=True)`` (nothing in a file is executed).
"""
import io
import os
import zipfile
from collections import OrderedDict
from typing import Any, Dict, List, Optional

import torch

TABLE_KEYS = ("mf_embedding_collection.embedding_bags.user_id.weight",
              "mf_embedding_collection.embedding_bags.product_id.weight",
              "mlp_embedding_collection.embedding_bags.user_id.weight",
              "mlp_embedding_collection.embedding_bags.product_id.weight")


def _optimizer_state(model, optimizer):
    from .trainer import FusedTrainStep
    if isinstance(optimizer, FusedTrainStep):
        opt = torch.optim.Adam(model.parameters(), lr=optimizer.lr, betas=optimizer.betas,
                               eps=optimizer.eps, weight_decay=optimizer.wd)
        optimizer.export_optimizer_state(opt)
        return opt.state_dict()
    return optimizer.state_dict()


def save_checkpoint(path: str, model, optimizer, epoch: int, metrics: Optional[Dict] = None,
                    config: Optional[Dict] = None, scheduler=None) -> str:
    """ModelTrainer._save_checkpoint (trainer.py:548-585)."""
    ckpt = {
        "epoch": epoch,
        "model_state_dict": model.state_dict(),
        "optimizer_state_dict": _optimizer_state(model, optimizer),
        "metrics": metrics,
        "config": config,
        "model_config": {"num_users": model.num_users, "num_products": model.num_products,
                         "embedding_dim": model.mf_embedding_dim},
    }
    if scheduler is not None:
        ckpt["scheduler_state_dict"] = scheduler.state_dict()
    torch.save(ckpt, path)
    return path


def load_checkpoint(path: str, model, optimizer=None, scheduler=None, map_location=None) -> int:
    """ModelTrainer._load_checkpoint (trainer.py:587-609): restores the model (strict), the
    optimizer and the scheduler when given; returns the next epoch."""
    from .trainer import FusedTrainStep
    dev = map_location or next(model.parameters()).device
    ckpt = torch.load(path, map_location=dev, weights_only=True)
    model.load_state_dict(ckpt["model_state_dict"])
    if optimizer is not None:
        if isinstance(optimizer, FusedTrainStep):
            optimizer.load_optimizer_state(ckpt["optimizer_state_dict"])
        else:
            optimizer.load_state_dict(ckpt["optimizer_state_dict"])
    if scheduler is not None and "scheduler_state_dict" in ckpt:
        scheduler.load_state_dict(ckpt["scheduler_state_dict"])
    return int(ckpt["epoch"]) + 1


def save_model(path: str, model) -> str:
    """Bare state_dict artifact (src/train.py:86-91)."""
    torch.save(model.state_dict(), path)
    return path


def load_model(path: str, model, strict: bool = True, map_location=None):
    """Load a bare state_dict file, or an unzipped torch.save directory, into ``model``."""
    dev = map_location or next(model.parameters()).device
    sd = (load_unzipped_archive(path, map_location=dev) if os.path.isdir(path)
          else torch.load(path, map_location=dev, weights_only=True))
    return model.load_state_dict(sd, strict=strict)


def load_unzipped_archive(directory: str, map_location="cpu") -> Any:
    """Read a ``torch.save`` zip archive that was extracted into ``directory`` (data.pkl,
    data/<key>, version, byteorder, .data/...) by zipping it back in memory and loading it with
    ``weights_only=True``: keys, shapes, strides and storage sharing come from the archive
    itself (consolidate_shards.py instead guesses them from raw tensor sizes)."""
    if not os.path.isfile(os.path.join(directory, "data.pkl")):
        raise FileNotFoundError(f"{directory}: no data.pkl (not an unzipped torch.save archive)")
    buf = io.BytesIO()
    with zipfile.ZipFile(buf, "w", zipfile.ZIP_STORED) as z:
        for root, _, files in os.walk(directory):
            for f in sorted(files):
                full = os.path.join(root, f)
                z.write(full, os.path.join("archive", os.path.relpath(full, directory)))
    buf.seek(0)
    return torch.load(buf, map_location=map_location, weights_only=True)


def consolidate_row_shards(shards: List[Dict[str, torch.Tensor]], world: int,
                           num_users: int, num_products: int) -> "OrderedDict[str, torch.Tensor]":
    """One full state_dict from the W ranks' state_dicts of the row-sharded step: table rows
    interleave (rank r holds ids r, r + W, ...); every other entry is replicated (rank 0's)."""
    if len(shards) != world:
        raise ValueError(f"expected {world} shards, got {len(shards)}")
    out = OrderedDict()
    for k, v in shards[0].items():
        if k in TABLE_KEYS:
            rows = num_users if ".user_id." in k else num_products
            full = torch.empty(rows, v.shape[1], dtype=v.dtype)
            for r in range(world):
                part = shards[r][k].cpu()
                full[r::world] = part[:len(range(r, rows, world))]
            out[k] = full
        else:
            out[k] = v.cpu().clone()
    return out


def shard_state_dict(full: Dict[str, torch.Tensor], world: int, rank: int):
    """Rank ``rank``'s state_dict of the row-sharded step from a full one (local tables of
    ceil(rows / W) rows, as make_sharded_step builds them; the padding rows are never read)."""
    out = OrderedDict()
    for k, v in full.items():
        if k in TABLE_KEYS:
            rows = v.shape[0]
            t = torch.zeros((rows + world - 1) // world, v.shape[1], dtype=v.dtype)
            own = v[rank::world]
            t[:own.shape[0]] = own
            out[k] = t
        else:
            out[k] = v.clone()
    return out
