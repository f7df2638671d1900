"""Checkpoint I/O with the reference's file names and schema.

* ``latest.pt`` = ``{'model','optimizer','scheduler','acc','epoch','step'}``
  written on suspend (reference ``restnet_ddp.py:37-44``), plus the optional
  superset key ``'scaler'`` for AMP (quirk Q9: the reference never saved it).
* ``best.pt`` = bare model ``state_dict`` (reference ``restnet_ddp.py:150``).

Model state is always torchvision layout (OIHW conv weights, torchvision key
names) even though the native engine keeps conv weights channels-last in a
flat buffer: ``state_dict()`` of the model already returns those views, and
``torch.save`` stores them with their logical shape. Writes are atomic (tmp +
rename) so a preemption mid-write never corrupts ``latest.pt``. Loads use
``weights_only=True``.
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import Any, Dict, Optional

import torch

__all__ = ["save_atomic", "save_latest", "load_latest", "save_best", "LATEST", "BEST"]

LATEST = "latest.pt"
BEST = "best.pt"


def _plain(sd):
    """Detach tensors to contiguous CPU copies so files are layout-independent."""
    if isinstance(sd, torch.Tensor):
        return sd.detach().to("cpu").contiguous().clone()
    if isinstance(sd, dict):
        return type(sd)((k, _plain(v)) for k, v in sd.items()) if not hasattr(sd, "_metadata") \
            else _with_meta(sd)
    if isinstance(sd, list):
        return [_plain(v) for v in sd]
    return sd


def _with_meta(sd):
    out = type(sd)((k, _plain(v)) for k, v in sd.items())
    out._metadata = getattr(sd, "_metadata", None)
    return out


def save_atomic(obj: Any, path) -> None:
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    tmp = path.with_name(path.name + f".tmp{os.getpid()}")
    torch.save(_plain(obj), tmp)
    os.replace(tmp, path)


def save_latest(save_path, model_sd, optimizer_sd, scheduler_sd, acc, epoch, step,
                scaler_sd: Optional[dict] = None) -> Path:
    state: Dict[str, Any] = {
        "model": model_sd,
        "optimizer": optimizer_sd,
        "scheduler": scheduler_sd,
        "acc": acc,
        "epoch": epoch,
        "step": step,
    }
    if scaler_sd is not None:
        state["scaler"] = scaler_sd
    p = Path(save_path) / LATEST
    save_atomic(state, p)
    return p


def load_latest(save_path) -> Optional[dict]:
    p = Path(save_path) / LATEST
    if not p.exists():
        return None
    return torch.load(p, map_location="cpu", weights_only=True)


def save_best(save_path, model_sd) -> Path:
    p = Path(save_path) / BEST
    save_atomic(model_sd, p)
    return p
