"""Real-image data path: ImageNet-style folder dataset + the reference's transforms.

The reference reads ImageNet through ``hfai.datasets.ImageNet`` (ffrecord) and
applies, for training, ``RandomResizedCrop(224) -> RandomHorizontalFlip() ->
ToTensor() -> Normalize(mean, std)`` and, for validation, ``Resize(256) ->
CenterCrop(224) -> ToTensor() -> Normalize`` (reference ``restnet_ddp.py:101-116``).
torchvision is not available, so the transforms are re-implemented on PIL +
numpy with the same parameters (scale (0.08, 1), ratio (3/4, 4/3), 10 attempts,
bilinear resampling, center-crop fallback).

Layout: ``<root>/<split>/<class_name>/*.{jpg,jpeg,png,...}``; classes are sorted
by name (``ImageFolder`` convention). Selected with ``MX_DATA=folder:<root>``.
Decoding runs in ``num_workers`` DataLoader worker processes with pinned
memory, as in the reference; the native engine converts the NCHW batch to its
space-to-depth layout on the GPU.
"""
from __future__ import annotations

import math
import os
import random
from typing import Callable, Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .synthetic import MEAN, STD

__all__ = ["ImageFolder", "train_transform", "val_transform", "FolderLoader"]

_EXT = (".jpg", ".jpeg", ".png", ".bmp", ".ppm", ".webp", ".tif", ".tiff")


def _to_tensor_normalized(img) -> torch.Tensor:
    a = np.asarray(img.convert("RGB"), dtype=np.float32) / 255.0
    a = (a - np.asarray(MEAN, dtype=np.float32)) / np.asarray(STD, dtype=np.float32)
    return torch.from_numpy(np.ascontiguousarray(a.transpose(2, 0, 1)))


def train_transform(size: int = 224, scale=(0.08, 1.0), ratio=(3 / 4, 4 / 3),
                    rng: Optional[random.Random] = None) -> Callable:
    rng = rng or random.Random()

    def f(img):
        from PIL import Image
        W, H = img.size
        area = W * H
        log_r = (math.log(ratio[0]), math.log(ratio[1]))
        box = None
        for _ in range(10):
            target = area * rng.uniform(*scale)
            ar = math.exp(rng.uniform(*log_r))
            w = int(round(math.sqrt(target * ar)))
            h = int(round(math.sqrt(target / ar)))
            if 0 < w <= W and 0 < h <= H:
                i = rng.randint(0, H - h)
                j = rng.randint(0, W - w)
                box = (j, i, j + w, i + h)
                break
        if box is None:  # fallback: center crop at the clamped ratio
            in_ratio = W / H
            if in_ratio < ratio[0]:
                w, h = W, int(round(W / ratio[0]))
            elif in_ratio > ratio[1]:
                h, w = H, int(round(H * ratio[1]))
            else:
                w, h = W, H
            i, j = (H - h) // 2, (W - w) // 2
            box = (j, i, j + w, i + h)
        img = img.resize((size, size), Image.BILINEAR, box=box)
        if rng.random() < 0.5:
            img = img.transpose(Image.FLIP_LEFT_RIGHT)
        return _to_tensor_normalized(img)

    return f


def val_transform(size: int = 224, resize: int = 256) -> Callable:
    def f(img):
        from PIL import Image
        W, H = img.size
        if W <= H:
            nw, nh = resize, int(resize * H / W)
        else:
            nh, nw = resize, int(resize * W / H)
        img = img.resize((nw, nh), Image.BILINEAR)
        top = int(round((nh - size) / 2.0))
        left = int(round((nw - size) / 2.0))
        img = img.crop((left, top, left + size, top + size))
        return _to_tensor_normalized(img)

    return f


class ImageFolder(torch.utils.data.Dataset):
    def __init__(self, root: str, split: str = "train", transform: Optional[Callable] = None) -> None:
        d = os.path.join(root, split)
        if not os.path.isdir(d):
            raise FileNotFoundError(f"no '{split}' split under {root}")
        self.classes = sorted(e for e in os.listdir(d) if os.path.isdir(os.path.join(d, e)))
        self.class_to_idx = {c: i for i, c in enumerate(self.classes)}
        self.samples: List[Tuple[str, int]] = []
        for c in self.classes:
            cd = os.path.join(d, c)
            for fn in sorted(os.listdir(cd)):
                if fn.lower().endswith(_EXT):
                    self.samples.append((os.path.join(cd, fn), self.class_to_idx[c]))
        if not self.samples:
            raise FileNotFoundError(f"no images under {d}")
        self.transform = transform
        self.split = split

    def __len__(self) -> int:
        return len(self.samples)

    def __getitem__(self, i: int):
        from PIL import Image
        path, label = self.samples[i]
        with open(path, "rb") as fh:
            img = Image.open(fh)
            img.load()
        x = self.transform(img) if self.transform else _to_tensor_normalized(img)
        return x, label

    def loader(self, batch_size: int, sampler=None, num_workers: int = 4, pin_memory: bool = True,
               max_steps: Optional[int] = None, **_) -> "FolderLoader":
        return FolderLoader(self, batch_size, sampler, num_workers, pin_memory, max_steps)


class _Slice(torch.utils.data.Sampler):
    def __init__(self, indices: Sequence[int]) -> None:
        self.indices = list(indices)

    def __iter__(self):
        return iter(self.indices)

    def __len__(self) -> int:
        return len(self.indices)


class FolderLoader:
    """DataLoader wrapper with the same ``iter_from`` / ``len`` contract as the synthetic loader."""

    def __init__(self, ds: ImageFolder, batch_size: int, sampler, num_workers: int, pin_memory: bool,
                 max_steps: Optional[int]) -> None:
        self.ds, self.batch_size, self.sampler = ds, batch_size, sampler
        self.num_workers, self.pin_memory, self.max_steps = num_workers, pin_memory, max_steps

    def _indices(self) -> List[int]:
        if self.sampler is None:
            return list(range(len(self.ds)))
        return list(iter(self.sampler))

    def __len__(self) -> int:
        n = math.ceil(len(self._indices()) / self.batch_size)
        return n if self.max_steps is None else min(n, self.max_steps)

    def iter_from(self, start_step: int = 0) -> Iterator:
        idx = self._indices()[start_step * self.batch_size:len(self) * self.batch_size]
        dl = torch.utils.data.DataLoader(self.ds, batch_size=self.batch_size, sampler=_Slice(idx),
                                         num_workers=self.num_workers, pin_memory=self.pin_memory
                                         and torch.cuda.is_available(),
                                         persistent_workers=False)
        for k, batch in enumerate(dl):
            yield start_step + k, batch

    def __iter__(self):
        for _, b in self.iter_from(0):
            yield b
