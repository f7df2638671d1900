"""``hfai.nccl.distributed`` equivalent (reference ``restnet_ddp.py:15``): the ``torch.distributed``
calls the reference makes -- ``init_process_group(backend, init_method, world_size, rank)``,
``get_rank``, ``get_world_size``, ``reduce``, ``all_reduce``, ``broadcast``, ``barrier`` -- with backend
``"nccl"`` meaning RCCL over xGMI on MI355X. On a host without a GPU ``"nccl"`` falls back to gloo,
so the same script runs in CPU tests."""
from __future__ import annotations

import torch
import torch.distributed as _dist
from torch.distributed import (ReduceOp, all_reduce, barrier, broadcast, destroy_process_group,  # noqa: F401
                               get_rank, get_world_size, is_initialized, reduce)

__all__ = ["init_process_group", "get_rank", "get_world_size", "reduce", "all_reduce", "broadcast",
           "barrier", "destroy_process_group", "is_initialized", "ReduceOp"]


def init_process_group(backend: str = "nccl", init_method=None, world_size: int = -1, rank: int = -1,
                       **kw):
    if backend == "nccl" and not torch.cuda.is_available():
        backend = "gloo"
    return _dist.init_process_group(backend=backend, init_method=init_method, world_size=world_size,
                                    rank=rank, **kw)
