"""DistributedDataParallel (replacement for ``hfai.nn.parallel.DistributedDataParallel``).

Reference usage: ``DistributedDataParallel(model.cuda(), device_ids=[local_rank])``
(``restnet_ddp.py:99``) and ``DistributedDataParallel(model)`` (``resnet_ddp_apex.py:103``).
Semantics kept from torch DDP (which the reference inherits):

* M2: parameters and buffers broadcast from rank 0 at construction;
* M4: buffers (BN running stats) broadcast from rank 0 before every
  grad-enabled forward (``broadcast_buffers=True``);
* M5: gradients averaged across ranks by bucketed all-reduce overlapping backward;
* ``.module`` exposes the wrapped model.

With the native model (:class:`~pytorch_distributed_amd.models.native.NativeResNet`)
parameters/gradients/buffers already live in flat buffers, so M2/M4 are ONE
broadcast each and M5 uses slices of the flat gradient as buckets, fired from
the native backward schedule (see :class:`NativeReducer`).
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import torch
from torch import nn

from .comm import Communicator, make_communicator
from .reducer import MiB, Reducer, plan_buckets

__all__ = ["DistributedDataParallel", "NativeReducer", "convert_sync_batchnorm"]


class NativeReducer:
    """Bucketed all-reduce over slices of a native model's flat gradient buffer.

    The native backward calls :meth:`grads_ready` with the number of leading
    elements of the flat gradient that are final (the flat buffer is laid out in
    gradient-production order). Each bucket whose end is covered is launched on
    the communicator stream immediately; :meth:`finish` makes the compute stream
    wait for all of them.
    """

    def __init__(self, flat_grad: torch.Tensor, boundaries: Sequence[int], comm: Communicator,
                 bucket_cap_mb: float = 32.0, first_bucket_mb: float = 1.0,
                 last_bucket_mb: Optional[float] = 2.0) -> None:
        self.flat = flat_grad
        self.comm = comm
        # boundaries: cumulative element offsets at which gradient segments complete
        segs = []
        prev = 0
        for b in boundaries:
            if b > prev:
                segs.append((prev, b))
                prev = b
        es = flat_grad.element_size()
        groups = plan_buckets([(e - s) * es for s, e in segs], int(bucket_cap_mb * MiB),
                              int(first_bucket_mb * MiB),
                              int(last_bucket_mb * MiB) if last_bucket_mb else None)
        self.buckets = [(segs[g[0]][0], segs[g[-1]][1]) for g in groups]
        self._next = 0
        self._works: List = []
        self.prescale = True
        # RCCL communicator: the bucket state machine runs in C++ (csrc/comm/reducer.cpp);
        # PDA_CPP_REDUCER=0 keeps the Python loop below (A/B, and the gloo/CPU communicators)
        self.native = None
        if (hasattr(comm, "make_bucket_reducer") and flat_grad.is_cuda
                and os.environ.get("PDA_CPP_REDUCER", "1") != "0"):
            self.native = comm.make_bucket_reducer(flat_grad, self.buckets)

    def reset(self) -> None:
        self._next = 0
        self._works = []
        if self.native is not None:
            self.native.reset()

    def grads_ready(self, upto: int) -> None:
        if self.native is not None:
            self.native.ready(upto)
            return
        while self._next < len(self.buckets) and self.buckets[self._next][1] <= upto:
            s, e = self.buckets[self._next]
            view = self.flat[s:e]
            if getattr(self.comm, "supports_avg", False):
                # RCCL ncclAvg: the 1/world scaling happens inside the collective (no extra pass)
                self._works.append(self.comm.all_reduce_async(view, op="avg"))
            else:
                if self.prescale and self.comm.world_size > 1:
                    view.div_(self.comm.world_size)
                self._works.append(self.comm.all_reduce_async(view))
            self._next += 1

    def finish(self) -> None:
        if self.native is not None:
            self.native.finish()
            return
        self.grads_ready(self.flat.numel())
        for w in self._works:
            self.comm.wait(w)
        self.reset()


def convert_sync_batchnorm(module: nn.Module, process_group=None) -> nn.Module:
    """``torch.nn.SyncBatchNorm.convert_sync_batchnorm`` counterpart (optional, off by
    default -- the reference keeps per-GPU statistics). A native model is flagged and, once
    wrapped in :class:`DistributedDataParallel`, all-reduces its BatchNorm sums (forward
    Σx/Σx², backward Σdz/Σdz·y) over a dedicated communicator before every finalize; a plain
    torch model gets ``nn.SyncBatchNorm`` layers."""
    if hasattr(module, "set_sync_bn"):
        module.sync_bn = True
        return module
    return nn.SyncBatchNorm.convert_sync_batchnorm(module, process_group)


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, device_ids: Optional[List[int]] = None,
                 output_device=None, broadcast_buffers: bool = True,
                 bucket_cap_mb: Optional[float] = None, process_group=None,
                 comm: Optional[Communicator] = None, sync_bn: Optional[bool] = None) -> None:
        super().__init__()
        self.module = module
        self.broadcast_buffers = broadcast_buffers
        dev = next(module.parameters()).device
        self.comm = comm if comm is not None else make_communicator(dev, process_group)
        # failure detection: poll the RCCL communicator's async error state from a
        # daemon thread; a dead peer aborts the communicator so collectives return (and the next
        # bucket wait raises) instead of hanging the job. MX_WATCHDOG=0 disables.
        if hasattr(self.comm, "start_watchdog") and os.environ.get("MX_WATCHDOG", "1") != "0":
            self.comm.start_watchdog(float(os.environ.get("MX_WATCHDOG_S", "5")))
        self._native = hasattr(module, "flat_params")
        cap = bucket_cap_mb or 32.0
        if self._native:
            module.sync_from_rank0(self.comm)                    # M2: one flat broadcast
            self.reducer = NativeReducer(module.flat_grad, module.grad_boundaries(), self.comm, cap)
            module.attach_reducer(self.reducer)
            self.bn_comm = None
            if (sync_bn if sync_bn is not None else getattr(module, "sync_bn", False)) \
                    and self.comm.world_size > 1:
                # SyncBN collectives run on the compute stream while bucket all-reduces run on
                # the comm stream: a second RCCL communicator keeps the two sequences independent
                self.bn_comm = (make_communicator(dev, process_group)
                                if hasattr(self.comm, "make_bucket_reducer") else self.comm)
                module.set_sync_bn(self.bn_comm)
        else:
            with torch.no_grad():
                for t in list(module.parameters()) + list(module.buffers()):   # M2
                    self.comm.broadcast(t.data, 0)
            self.reducer = Reducer(module.parameters(), self.comm, cap)

    def _sync_buffers(self) -> None:
        if self._native:
            self.module.broadcast_buffers_from_rank0(self.comm)
            return
        with torch.no_grad():
            for b in self.module.buffers():
                self.comm.broadcast(b.data, 0)

    def forward(self, *args, **kwargs):
        if self.broadcast_buffers and self.module.training and torch.is_grad_enabled() \
                and self.comm.world_size > 1:
            self._sync_buffers()                                      # M4
        return self.module(*args, **kwargs)

    def state_dict(self, *a, **k):
        return super().state_dict(*a, **k)
