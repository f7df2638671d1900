"""``hfai.datasets.ImageNet`` equivalent (reference ``restnet_ddp.py:107,117``).

``ImageNet(split, transform=None)`` returns a dataset whose ``.loader(batch_size, sampler=None,
num_workers=4, pin_memory=True)`` yields ``(samples, labels)`` batches with ``len()`` -- the contract
the reference's ``train``/``validate`` rely on. With ``MX_DATA=folder:<root>`` (or ``root=``) it reads
an ImageNet-style folder through PIL with ``transform`` applied per image; otherwise it is the
synthetic ImageNet (1,281,167 / 50,000 virtual samples, already normalised, so ``transform`` --
written for PIL images -- does not apply and is ignored).
"""
from __future__ import annotations

import os
from typing import Callable, Optional

from ..data.folder import ImageFolder
from ..data.synthetic import SyntheticImageNet

__all__ = ["ImageNet"]


def ImageNet(split: str, transform: Optional[Callable] = None, root: Optional[str] = None,
             image_size: Optional[int] = None, num_samples: Optional[int] = None):
    data = os.environ.get("MX_DATA", "synthetic")
    if root is None and data.startswith("folder:"):
        root = data.split(":", 1)[1]
    if root is not None:
        return ImageFolder(root, split, transform)
    size = image_size or int(os.environ.get("MX_IMAGE_SIZE", "224"))
    return SyntheticImageNet(split, num_samples=num_samples, image_size=size)
