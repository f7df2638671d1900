"""Single-process multi-GPU data parallel (replacement for ``nn.DataParallel``).

Reference: ``nn.DataParallel(model.cuda(), device_ids=gpus, output_device=gpus[0])``
(``resnet_dp.py:82``) with a 3200-sample global batch. torch's implementation
(``torch/nn/parallel/data_parallel.py:173-198``) re-replicates the module from
GPU0 every step (13 coalesced 10 MiB broadcasts), runs replicas in Python
threads, gathers logits on GPU0 and reduce-adds gradients to GPU0;
that is why the reference's DP reaches only 59.8% GPU utilisation.

This implementation keeps the API and the math (replica 0 owns the parameters
and the optimizer; BN running stats follow replica 0; outputs gathered on
``output_device``) but:

* replicas are *persistent* -- created once, refreshed each forward by one
  broadcast of replica 0's parameters+buffers (a single flat buffer for native
  models) instead of rebuilding modules;
* gradients are summed into replica 0 by one reduce over the flat gradient at
  the end of backward (queued autograd callback), not per-parameter chunks.
"""
from __future__ import annotations

import copy
from typing import List, Optional, Sequence

import torch
from torch import nn

__all__ = ["DataParallel"]


class _Gather(torch.autograd.Function):
    @staticmethod
    def forward(ctx, dst, *outs):
        ctx.devices = [o.device for o in outs]
        ctx.sizes = [o.shape[0] for o in outs]
        return torch.cat([o.to(dst, non_blocking=True) for o in outs], 0)

    @staticmethod
    def backward(ctx, g):
        parts = torch.split(g, ctx.sizes, 0)
        return (None,) + tuple(p.to(d, non_blocking=True) for p, d in zip(parts, ctx.devices))


class DataParallel(nn.Module):
    def __init__(self, module: nn.Module, device_ids: Optional[Sequence[int]] = None,
                 output_device=None, dim: int = 0) -> None:
        super().__init__()
        self.module = module
        dev = next(module.parameters()).device
        if dev.type != "cuda":
            device_ids = []
        elif device_ids is None:
            device_ids = list(range(torch.cuda.device_count()))
        self.device_ids = [int(d) for d in device_ids]
        self.output_device = self.device_ids[0] if output_device is None and self.device_ids \
            else output_device
        self.replicas: List[nn.Module] = []
        for d in self.device_ids[1:]:
            if hasattr(module, "replicate_to"):
                self.replicas.append(module.replicate_to(torch.device("cuda", d)))
            else:
                self.replicas.append(copy.deepcopy(module).to(torch.device("cuda", d)))
        self._armed = False

    # -- parameter/grad sync -------------------------------------------------------------
    @torch.no_grad()
    def _broadcast_params(self) -> None:
        if not self.replicas:
            return
        src = list(self.module.parameters()) + list(self.module.buffers())
        for r in self.replicas:
            dst = list(r.parameters()) + list(r.buffers())
            for s, t in zip(src, dst):
                t.copy_(s, non_blocking=True)

    @torch.no_grad()
    def _reduce_grads(self) -> None:
        self._armed = False
        for r in self.replicas:
            for p0, pr in zip(self.module.parameters(), r.parameters()):
                if pr.grad is None:
                    continue
                g = pr.grad.to(p0.device, non_blocking=True)
                if p0.grad is None:
                    p0.grad = g.clone()
                else:
                    p0.grad.add_(g)
                pr.grad = None

    def train(self, mode: bool = True):
        super().train(mode)
        for r in self.replicas:
            r.train(mode)
        return self

    def forward(self, x: torch.Tensor, *args, **kwargs):
        if not self.replicas:
            return self.module(x, *args, **kwargs)
        self._broadcast_params()
        chunks = torch.chunk(x, len(self.device_ids), 0)
        outs = []
        mods = [self.module] + self.replicas
        for m, c, d in zip(mods, chunks, self.device_ids):
            with torch.cuda.device(d):
                outs.append(m(c.to(torch.device("cuda", d), non_blocking=True), *args, **kwargs))
        if torch.is_grad_enabled() and not self._armed:
            self._armed = True
            out = _Gather.apply(torch.device("cuda", self.output_device), *outs)
            out.register_hook(self._arm_callback)
            return out
        return torch.cat([o.to(torch.device("cuda", self.output_device)) for o in outs], 0)

    def _arm_callback(self, g):
        torch.autograd.Variable._execution_engine.queue_callback(self._reduce_grads)
        return g
