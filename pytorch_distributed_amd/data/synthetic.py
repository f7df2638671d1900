"""Synthetic ImageNet: deterministic virtual samples generated on the fly.

Replaces the reference's ffrecord ``hfai.datasets.ImageNet`` + 4-worker
JPEG-decoding ``DataLoader`` (reference ``restnet_ddp.py:101-119``,
SURVEY §2.3 X2) so that runs need no dataset.

Every sample ``i`` of a split is a pure function of ``(seed, split, i)``:

* label  = ``hash32(i, seed, split) % num_classes``
* pixel  = ``(u + 0.5 * class_tint[label, c] - mean[c]) / std[c]`` where ``u`` in
  [0,1) is ``hash32`` of the element coordinates -- i.e. already in the
  ``ToTensor() + Normalize(mean, std)`` range of the reference transforms, with a
  label-dependent colour tint so a model can actually learn (loss decreases).

The same integer hash is implemented in torch here (CPU / reference path) and
in HIP (``csrc/kernels/data.hip``, on-device NHWC generation), and the two are
bit-compatible in the label and the uniform ``u`` (tested).
"""
from __future__ import annotations

import math
from typing import Iterator, Optional, Tuple

import torch

from .sampler import SequentialIndices

__all__ = [
    "MEAN", "STD", "hash32", "labels_for", "synthetic_images", "SyntheticImageNet",
    "BatchLoader",
]

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)
_M32 = 0xFFFFFFFF
SPLIT_ID = {"train": 1, "val": 2}


def hash32(x: torch.Tensor) -> torch.Tensor:
    """lowbias32 integer hash on int64 tensors holding uint32 values."""
    x = x & _M32
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    x = x ^ (x >> 16)
    return x


def _sample_key(ids: torch.Tensor, seed: int, split: str) -> torch.Tensor:
    return hash32(ids.to(torch.int64) * 2654435761 + (seed * 97 + SPLIT_ID[split]) * 0x632BE5AB)


def labels_for(ids: torch.Tensor, seed: int, split: str, num_classes: int) -> torch.Tensor:
    return hash32(_sample_key(ids, seed, split) ^ 0x5BD1E995) % num_classes


def class_tint(labels: torch.Tensor, c: int) -> torch.Tensor:
    """Per-(class, channel) tint in {0, 1/3, 2/3, 1}."""
    return ((labels * (2 * c + 3) + c) % 4).to(torch.float32) / 3.0


def synthetic_images(ids: torch.Tensor, seed: int, split: str, num_classes: int,
                     image_size: int = 224, device=None,
                     dtype: torch.dtype = torch.float32) -> Tuple[torch.Tensor, torch.Tensor]:
    """Generate ``(images[B,3,S,S] NCHW, labels[B])`` with torch ops (any device)."""
    device = ids.device if device is None else torch.device(device)
    ids = ids.to(device=device, dtype=torch.int64)
    key = _sample_key(ids, seed, split)                       # [B]
    labels = hash32(key ^ 0x5BD1E995) % num_classes
    hw = image_size * image_size
    pos = torch.arange(3 * hw, device=device, dtype=torch.int64)  # (c, y, x) flattened
    u = hash32(key[:, None] ^ (pos[None, :] * 0x27D4EB2F))
    u = (u >> 8).to(torch.float32) * (1.0 / 16777216.0)        # [B, 3*hw] in [0,1)
    u = u.view(-1, 3, image_size, image_size)
    out = torch.empty_like(u)
    for c in range(3):
        tint = class_tint(labels, c).view(-1, 1, 1)
        out[:, c] = (u[:, c] * 0.5 + 0.5 * tint - MEAN[c]) / STD[c]
    return out.to(dtype), labels


class SyntheticImageNet:
    """Map-style dataset of virtual ImageNet samples (train 1,281,167 / val 50,000)."""

    def __init__(self, split: str = "train", num_samples: Optional[int] = None, seed: int = 0,
                 num_classes: int = 1000, image_size: int = 224) -> None:
        if split not in SPLIT_ID:
            raise ValueError(split)
        self.split = split
        self.num_samples = num_samples if num_samples is not None else (
            1_281_167 if split == "train" else 50_000)
        self.seed = seed
        self.num_classes = num_classes
        self.image_size = image_size

    def __len__(self) -> int:
        return self.num_samples

    def __getitem__(self, i: int) -> Tuple[torch.Tensor, int]:
        x, y = synthetic_images(torch.tensor([i]), self.seed, self.split, self.num_classes,
                                self.image_size)
        return x[0], int(y[0])

    def batch(self, ids: torch.Tensor, device=None, dtype=torch.float32):
        return synthetic_images(ids, self.seed, self.split, self.num_classes, self.image_size,
                                device=device, dtype=dtype)

    def loader(self, batch_size: int, sampler=None, num_workers: int = 4, pin_memory: bool = True,
               device=None, generator=None, max_steps: Optional[int] = None) -> "BatchLoader":
        """Mirror of ``hfai.datasets.ImageNet(...).loader(...)`` (reference ``restnet_ddp.py:109``).

        ``num_workers``/``pin_memory`` are accepted for API parity; synthetic batches are
        produced directly on ``device`` (no host decode, no H2D copy).
        ``generator`` optionally overrides batch production (e.g. the native on-device
        NHWC kernel); it is called as ``generator(ids) -> (images, labels)``.
        """
        return BatchLoader(self, batch_size, sampler, device=device, generator=generator,
                           max_steps=max_steps)


class BatchLoader:
    """Iterable of ``(samples, labels)`` batches with ``len()`` (drop_last=False)."""

    def __init__(self, dataset: SyntheticImageNet, batch_size: int, sampler=None, device=None,
                 generator=None, max_steps: Optional[int] = None) -> None:
        self.dataset = dataset
        self.batch_size = batch_size
        self.sampler = sampler if sampler is not None else SequentialIndices(len(dataset))
        self.device = device
        self.generator = generator
        self.max_steps = max_steps
        self.start_step = 0

    def __len__(self) -> int:
        n = math.ceil(len(self.sampler) / self.batch_size)
        return n if self.max_steps is None else min(n, self.max_steps)

    def indices(self) -> torch.Tensor:
        return torch.as_tensor(list(iter(self.sampler)) if not hasattr(self.sampler, "index_tensor")
                               else self.sampler.index_tensor(), dtype=torch.int64)

    def batch_ids(self, step: int, idx: Optional[torch.Tensor] = None) -> torch.Tensor:
        idx = self.indices() if idx is None else idx
        return idx[step * self.batch_size:(step + 1) * self.batch_size]

    def iter_from(self, start_step: int = 0) -> Iterator[Tuple[int, Tuple[torch.Tensor, torch.Tensor]]]:
        """Yield ``(step, batch)`` beginning at ``start_step`` without generating the skipped
        batches (the reference iterates and discards them, quirk Q10; the resulting sample
        order is identical)."""
        idx = self.indices()
        for step in range(start_step, len(self)):
            ids = idx[step * self.batch_size:(step + 1) * self.batch_size]
            if self.generator is not None:
                yield step, self.generator(ids)
            else:
                yield step, self.dataset.batch(ids, device=self.device)

    def __iter__(self):
        for _, b in self.iter_from(0):
            yield b
