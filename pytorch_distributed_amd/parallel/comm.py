"""Communicator: the collective layer under DDP / DP / validation.

Two implementations behind one interface:

* :class:`RcclCommunicator` -- our C++ RCCL communicator (``csrc/comm/rccl_comm.cpp``):
  ``ncclGetUniqueId`` exchanged through the ``torch.distributed`` TCPStore,
  ``ncclCommInitRank``, collectives enqueued on a dedicated HIP stream that
  waits on an event recorded on the compute stream, completion tracked by a
  HIP event the compute stream later waits on (no host sync). Used for the
  gradient buckets on GPU.
* :class:`ProcessGroupCommunicator` -- any initialised ``torch.distributed``
  process group (``gloo`` on CPU for the multi-process CPU tests; ``nccl`` = RCCL
  on ROCm as a fallback when the native extension is unavailable).
"""
from __future__ import annotations

from typing import Any, Optional

import torch
import torch.distributed as dist

__all__ = ["Communicator", "ProcessGroupCommunicator", "make_communicator", "register_default",
           "default_communicator"]

# the process's device communicator per device (set by DistributedDataParallel on the default
# group): the hfai-compatible ``platform.nccl.distributed`` collectives use it, so a ported script
# calling ``dist.reduce`` does not create torch's NCCL communicator beside it
_DEFAULTS = {}


def register_default(comm: "Communicator", device: torch.device) -> None:
    _DEFAULTS[str(torch.device(device))] = comm


def default_communicator(device: torch.device) -> Optional["Communicator"]:
    c = _DEFAULTS.get(str(torch.device(device)))
    if c is not None and getattr(c, "aborted", False):
        return None
    return c


class Communicator:
    world_size: int = 1
    rank: int = 0

    def all_reduce_async(self, t: torch.Tensor) -> Any:
        raise NotImplementedError

    def wait(self, handle: Any) -> None:
        raise NotImplementedError

    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> None:
        if op != "sum":
            raise NotImplementedError(op)
        self.wait(self.all_reduce_async(t))

    def broadcast(self, t: torch.Tensor, src: int = 0) -> None:
        raise NotImplementedError

    def broadcast_async(self, t: torch.Tensor, src: int = 0) -> Any:
        """Broadcast that may complete later; the returned handle goes to :meth:`wait`. Default:
        synchronous (returns None)."""
        self.broadcast(t, src)
        return None

    def barrier(self) -> None:
        raise NotImplementedError


class ProcessGroupCommunicator(Communicator):
    def __init__(self, group=None) -> None:
        self.group = group
        self.world_size = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    def all_reduce_async(self, t: torch.Tensor):
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def wait(self, handle) -> None:
        if handle is not None:
            handle.wait()

    _OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}

    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> None:
        dist.all_reduce(t, op=self._OPS[op], group=self.group)

    def broadcast(self, t: torch.Tensor, src: int = 0) -> None:
        dist.broadcast(t, src=src, group=self.group)

    def barrier(self) -> None:
        dist.barrier(group=self.group)


def make_communicator(device: Optional[torch.device] = None, group=None,
                      prefer_native: bool = True) -> Communicator:
    """Native RCCL communicator on GPU when the extension is built, else process group."""
    import os
    prefer_native = prefer_native and os.environ.get("PDA_COMM", "native") == "native"
    if device is not None and device.type == "cuda" and prefer_native \
            and dist.get_backend(group) == "nccl":
        try:
            from .rccl import RcclCommunicator
            return RcclCommunicator(device, group=group)
        except (ImportError, RuntimeError) as e:  # pragma: no cover - GPU only
            import warnings
            warnings.warn(f"native RCCL communicator unavailable ({e}); using torch process group")
    return ProcessGroupCommunicator(group)
