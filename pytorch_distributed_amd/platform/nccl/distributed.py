"""``hfai.nccl.distributed`` equivalent (reference ``restnet_ddp.py:15``): the ``torch.distributed``
calls the reference makes -- ``init_process_group(backend, init_method, world_size, rank)``,
``get_rank``, ``get_world_size``, ``reduce``, ``all_reduce``, ``broadcast``, ``barrier`` -- with backend
``"nccl"`` meaning RCCL over xGMI on MI355X. On a host without a GPU ``"nccl"`` falls back to gloo,
so the same script runs in CPU tests.

Device collectives on the default group go through the process's own RCCL communicator once
:class:`~pytorch_distributed_amd.parallel.ddp.DistributedDataParallel` has created it
(:func:`~pytorch_distributed_amd.parallel.comm.default_communicator`), ordered on the current
stream: a ported script's ``dist.reduce(x, 0)`` of its validation counters
(``/root/reference/restnet_ddp.py:63-64``) then never creates torch's ProcessGroupNCCL communicator
beside the framework's (one RCCL communicator per process). Before a DDP exists, for a
``group`` argument, a non-contiguous tensor or an op the native communicator lacks (PRODUCT...),
the call is torch's."""
from __future__ import annotations

import torch
import torch.distributed as _dist
from torch.distributed import (ReduceOp, destroy_process_group, get_rank, get_world_size,  # noqa: F401
                               is_initialized)

__all__ = ["init_process_group", "get_rank", "get_world_size", "reduce", "all_reduce", "broadcast",
           "barrier", "destroy_process_group", "is_initialized", "ReduceOp"]

_OPS = {ReduceOp.SUM: "sum", ReduceOp.MAX: "max", ReduceOp.MIN: "min", ReduceOp.AVG: "avg"}


def init_process_group(backend: str = "nccl", init_method=None, world_size: int = -1, rank: int = -1,
                       **kw):
    if backend == "nccl" and not torch.cuda.is_available():
        backend = "gloo"
    return _dist.init_process_group(backend=backend, init_method=init_method, world_size=world_size,
                                    rank=rank, **kw)


class _Done:
    """``async_op=True`` handle of a native collective: it is stream-ordered, so waiting means
    nothing more than the current stream already guarantees."""

    def wait(self, timeout=None) -> bool:
        return True

    def is_completed(self) -> bool:
        return True


def _native(tensor: torch.Tensor, group, op=None):
    if group is not None or not isinstance(tensor, torch.Tensor) or not tensor.is_contiguous():
        return None
    if op is not None and op not in _OPS:
        return None
    from ...parallel.comm import default_communicator
    return default_communicator(tensor.device)


def reduce(tensor, dst, op=ReduceOp.SUM, group=None, async_op=False):
    c = _native(tensor, group, op)
    if c is None or not hasattr(c, "reduce"):
        return _dist.reduce(tensor, dst, op=op, group=group, async_op=async_op)
    c.reduce(tensor, dst, _OPS[op])
    return _Done() if async_op else None


def all_reduce(tensor, op=ReduceOp.SUM, group=None, async_op=False):
    c = _native(tensor, group, op)
    if c is None:
        return _dist.all_reduce(tensor, op=op, group=group, async_op=async_op)
    c.all_reduce(tensor, _OPS[op])
    return _Done() if async_op else None


def broadcast(tensor, src, group=None, async_op=False):
    c = _native(tensor, group)
    if c is None:
        return _dist.broadcast(tensor, src, group=group, async_op=async_op)
    c.broadcast(tensor, src)
    return _Done() if async_op else None


def barrier(group=None, async_op=False, device_ids=None):
    # host-side barrier: never on a device communicator (no GPU work to order)
    from ...launch import host_group
    g = group if group is not None else (host_group() if _dist.get_backend() != "gloo" else None)
    return _dist.barrier(group=g, async_op=async_op)
