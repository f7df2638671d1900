"""Index samplers.

:class:`DistributedSampler` reproduces ``torch.utils.data.DistributedSampler``
index math exactly (``torch/utils/data/distributed.py:107-134``; used by the
reference at ``restnet_ddp.py:108,118``): ``randperm`` seeded with
``seed + epoch``, padded to a multiple of ``world`` by repeating the head, then
``indices[rank::world]``. Quirk Q11 (padded duplicates in validation) is
therefore reproduced.
"""
from __future__ import annotations

import math
from typing import Iterator, Optional

import torch

__all__ = ["DistributedSampler", "SequentialIndices"]


class SequentialIndices:
    """Default sampler of a loader without ``sampler=`` (torch DataLoader: shuffle=False)."""

    def __init__(self, n: int) -> None:
        self.n = n

    def __len__(self) -> int:
        return self.n

    def index_tensor(self) -> torch.Tensor:
        return torch.arange(self.n, dtype=torch.int64)

    def __iter__(self) -> Iterator[int]:
        return iter(range(self.n))


class DistributedSampler:
    def __init__(self, dataset, num_replicas: Optional[int] = None, rank: Optional[int] = None,
                 shuffle: bool = True, seed: int = 0, drop_last: bool = False) -> None:
        if num_replicas is None or rank is None:
            import torch.distributed as dist
            if not dist.is_available() or not dist.is_initialized():
                raise RuntimeError("DistributedSampler needs an initialised process group "
                                   "or explicit num_replicas/rank")
            num_replicas = dist.get_world_size() if num_replicas is None else num_replicas
            rank = dist.get_rank() if rank is None else rank
        if not 0 <= rank < num_replicas:
            raise ValueError(f"invalid rank {rank} for world {num_replicas}")
        self.n = len(dataset)
        self.num_replicas = num_replicas
        self.rank = rank
        self.shuffle = shuffle
        self.seed = seed
        self.drop_last = drop_last
        self.epoch = 0
        if drop_last and self.n % num_replicas != 0:
            self.num_samples = math.ceil((self.n - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(self.n / num_replicas)
        self.total_size = self.num_samples * num_replicas

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch

    def __len__(self) -> int:
        return self.num_samples

    def index_tensor(self) -> torch.Tensor:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g)
        else:
            idx = torch.arange(self.n, dtype=torch.int64)
        if not self.drop_last:
            pad = self.total_size - idx.numel()
            if pad > 0:
                reps = math.ceil(pad / idx.numel())
                idx = torch.cat([idx, idx.repeat(reps)[:pad]])
        else:
            idx = idx[: self.total_size]
        assert idx.numel() == self.total_size
        return idx[self.rank:self.total_size:self.num_replicas]

    def __iter__(self) -> Iterator[int]:
        return iter(self.index_tensor().tolist())
