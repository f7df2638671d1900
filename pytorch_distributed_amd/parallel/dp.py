"""Single-process multi-GPU data parallel (replacement for ``nn.DataParallel``).

Reference: ``nn.DataParallel(model.cuda(), device_ids=gpus, output_device=gpus[0])``
(``resnet_dp.py:82``) with a 3200-sample global batch. torch's implementation
(``torch/nn/parallel/data_parallel.py:173-198``) re-replicates the module from
GPU0 every step (13 coalesced 10 MiB broadcasts), runs replicas in Python
threads, gathers logits on GPU0 and reduce-adds gradients to GPU0;
that is why the reference's DP reaches only 59.8% GPU utilisation.

This implementation keeps the API and the math (outputs gathered on
``output_device``; the loss is computed there over the global batch; BN running
statistics follow replica 0) but is built for a fully connected xGMI node:

* replicas are *persistent*. For the native engine each GPU holds a full
  :class:`~pytorch_distributed_amd.models.native.NativeResNet` (flat buffers);
* after backward the flat gradients are SUM-all-reduced across the local GPUs by
  ONE grouped in-process RCCL collective (``ncclCommInitAll`` communicator,
  :class:`~pytorch_distributed_amd.parallel.rccl.RcclGroup`), and every replica
  runs the fused SGD itself (replicated update: mathematically identical to
  reduce-to-GPU0 + step + broadcast, with no per-step weight broadcast);
* BN buffers (213 KB) are broadcast from replica 0 before each training forward,
  which is what torch's per-step ``replicate`` achieves for them.

For arbitrary (non-native) modules it falls back to persistent deep-copied
replicas with a parameter refresh before each forward and a gradient
reduction into replica 0 after backward -- the same math as ``nn.DataParallel``.
"""
from __future__ import annotations

import copy
from typing import List, Optional, Sequence

import torch
from torch import nn

__all__ = ["DataParallel", "ReplicatedSGD"]


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


class ReplicatedSGD(torch.optim.Optimizer):
    """One fused SGD per replica, stepped after the in-process gradient all-reduce. Exposes
    replica 0's ``param_groups`` / ``state_dict`` (what schedulers and checkpoints see)."""

    def __init__(self, opts) -> None:
        super().__init__(opts[0].param_groups[0]["params"], opts[0].defaults)
        self.opts = opts
        self.param_groups = opts[0].param_groups
        self.state = opts[0].state

    def _sync_hparams(self) -> None:
        for o in self.opts[1:]:
            for g0, g in zip(self.param_groups, o.param_groups):
                for k in ("lr", "momentum", "weight_decay"):
                    g[k] = g0[k]

    def zero_grad(self, set_to_none: bool = True) -> None:
        for o in self.opts:
            o.zero_grad(set_to_none)

    def step(self, closure=None):
        self._sync_hparams()
        for o in self.opts:
            with torch.cuda.device(o.model.device):
                o.step()

    def step_amp(self, scale, found_inf, tracker=None, growth_factor=2.0, backoff_factor=0.5,
                 growth_interval=2000):
        # every replica holds the same (all-reduced) gradient, so the inf check agrees; replica 0
        # owns the scaler state (its kernel updates scale/tracker), the others unscale with copies
        self._sync_hparams()
        # copies of the CURRENT scale first: replica 0's kernel updates it in place
        copies = [scale.to(o.model.device, copy=True) for o in self.opts[1:]]
        with torch.cuda.device(self.opts[0].model.device):
            self.opts[0].step_amp(scale, found_inf, tracker, growth_factor, backoff_factor,
                                  growth_interval)
        for o, s in zip(self.opts[1:], copies):
            with torch.cuda.device(o.model.device):
                o.step_amp(s, torch.zeros_like(found_inf, device=o.model.device))

    def state_dict(self):
        return self.opts[0].state_dict()

    def load_state_dict(self, sd):
        for o in self.opts:
            o.load_state_dict(copy.deepcopy(sd))
        self.param_groups = self.opts[0].param_groups
        self.state = self.opts[0].state


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
        if self.device_ids and dev.index != self.device_ids[0]:
            raise ValueError("module must live on device_ids[0]")
        self.output_device = self.device_ids[0] if (output_device is None and self.device_ids) \
            else output_device
        self._native = hasattr(module, "flat_params")
        self.replicas: List[nn.Module] = []
        self.group = None
        for d in self.device_ids[1:]:
            dd = torch.device("cuda", d)
            if self._native:
                self.replicas.append(self._native_replica(dd))
            else:
                self.replicas.append(copy.deepcopy(module).to(dd))
        if self._native and self.replicas and len(set(self.device_ids)) == len(self.device_ids):
            from .rccl import RcclGroup
            self.group = RcclGroup(self.device_ids)
        # (replicas sharing a device -- used by the 1-GPU tests -- sync through plain copies)
        self._armed = False

    # ------------------------------------------------------------------ construction
    def _native_replica(self, dev: torch.device):
        from ..models.native import NativeResNet
        from ..models.resnet import ResNet
        m = self.module
        ref = ResNet(m.arch_block, [len(getattr(m, f"layer{i}")) for i in range(1, 5)], m.num_classes)
        with torch.cuda.device(dev):
            r = NativeResNet(ref, device=dev, dtype=m.dtype, image_size=m.image_size)
            with torch.no_grad():
                r.flat_params.copy_(m.flat_params)
                r.flat_bufstore.copy_(m.flat_bufstore)
            r.refresh_shadow()
        return r

    @property
    def all_modules(self) -> List[nn.Module]:
        return [self.module] + self.replicas

    # ------------------------------------------------------------------ factories
    def make_optimizer(self, **kw):
        if self._native:
            opts = [m.make_optimizer(**kw) for m in self.all_modules]
            return ReplicatedSGD(opts) if self.replicas else opts[0]
        return torch.optim.SGD(self.module.parameters(), **kw)

    def make_criterion(self):
        if not self.replicas and hasattr(self.module, "make_criterion"):
            return self.module.make_criterion()
        return nn.CrossEntropyLoss()   # gathered logits: gradient flows back through _Gather

    def input_generator(self, ds):
        return self.module.input_generator(ds) if hasattr(self.module, "input_generator") else None

    # ------------------------------------------------------------------ sync
    @torch.no_grad()
    def _broadcast_state(self) -> None:
        if not self.replicas:
            return
        if self._native:
            ts = [m.flat_bufstore for m in self.all_modules]   # running stats + counters
            if self.group is not None:
                self.group.broadcast(ts, 0)
            else:
                for t in ts[1:]:
                    t.copy_(ts[0], non_blocking=True)
            return
        src = list(self.module.parameters()) + list(self.module.buffers())
        for r in self.replicas:
            for s, t in zip(src, list(r.parameters()) + list(r.buffers())):
                t.copy_(s, non_blocking=True)

    @torch.no_grad()
    def _reduce_grads(self) -> None:
        self._armed = False
        if self._native:
            ts = [m.flat_grad for m in self.all_modules]
            if self.group is not None:
                self.group.all_reduce(ts)
            else:
                total = ts[0].clone()
                for t in ts[1:]:
                    total.add_(t.to(total.device))
                for t in ts:
                    t.copy_(total, non_blocking=True)
            for m in self.all_modules:
                m._grads_zero = False
            return
        for r in self.replicas:
            for p0, pr in zip(self.module.parameters(), r.parameters()):
                if pr.grad is None:
                    continue
                g = pr.grad.to(p0.device, non_blocking=True)
                p0.grad = g.clone() if p0.grad is None else p0.grad.add_(g)
                pr.grad = None

    def zero_grad(self, set_to_none: bool = True) -> None:
        for m in self.all_modules:
            m.zero_grad(set_to_none)

    def train(self, mode: bool = True):
        super().train(mode)
        for r in self.replicas:
            r.train(mode)
        return self

    def state_dict(self, *a, **k):
        return self.module.state_dict(*a, **k)

    def load_state_dict(self, sd, strict: bool = True):
        res = self.module.load_state_dict(sd, strict=strict)
        if self._native:
            for r in self.replicas:
                r.load_state_dict(sd, strict=strict)
        return res

    # ------------------------------------------------------------------ forward
    def forward(self, x: torch.Tensor, *args, **kwargs):
        if not self.replicas:
            return self.module(x, *args, **kwargs)
        self._broadcast_state()
        chunks = torch.chunk(x, len(self.device_ids), 0)
        outs = []
        for m, c, d in zip(self.all_modules, chunks, self.device_ids):
            with torch.cuda.device(d):
                outs.append(m(c.to(torch.device("cuda", d), non_blocking=True), *args, **kwargs))
        if torch.is_grad_enabled() and outs[0].requires_grad:
            out = _Gather.apply(torch.device("cuda", self.output_device), *outs)
            out.register_hook(self._arm_callback)
            return out
        return torch.cat([o.to(torch.device("cuda", self.output_device)) for o in outs], 0)

    # ------------------------------------------------------------------ graph-replayed step
    def graph_step_ok(self, scaler=None) -> bool:
        """The HIP-graph step serves the native engine without loss scaling (the DP script's
        configuration). ``MX_GRAPH=0`` forces the eager autograd path."""
        import os
        return (self._native and bool(self.device_ids) and (scaler is None or not scaler.enabled)
                and os.environ.get("MX_GRAPH", "1") != "0")

    def train_step(self, samples: torch.Tensor, labels: torch.Tensor, optimizer,
                   graph: bool = True) -> torch.Tensor:
        """One DP training step with every replica's forward + loss + backward replayed from a HIP
        graph: ONE host launch per device instead of ~600 (the eager schedule costs ~8 ms of host
        time per device per ResNet-50 step, so one thread driving 8 GPUs eagerly would be
        launch-bound; see ``tools/host_overhead.py``). Same math as ``crit(dp(x), y).backward();
        optimizer.step()``: the loss is the mean over the GLOBAL batch (each replica's gradient
        is scaled by 1/B_global), BN statistics are per replica, BN buffers follow replica 0,
        gradients are SUM-all-reduced by one grouped RCCL call, then the replicated fused SGD."""
        xs = torch.chunk(samples, len(self.device_ids), 0)
        ys = torch.chunk(labels, len(self.device_ids), 0)
        return self.train_step_chunks(xs, ys, optimizer, graph)

    def train_step_chunks(self, xs, ys, optimizer, graph: bool = True) -> torch.Tensor:
        """:meth:`train_step` on per-replica input chunks (e.g. generated on each GPU directly,
        skipping the scatter from ``device_ids[0]``)."""
        self._broadcast_state()
        B = sum(x.shape[0] for x in xs)
        if getattr(self, "_graphs", None) is None or [x.shape for x in xs] != self._graph_shapes:
            self._graphs = [_ReplicaGraph(m, x.shape, B) for m, x in zip(self.all_modules, xs)]
            self._graph_shapes = [x.shape for x in xs]
        jobs = list(zip(self._graphs, xs, ys))
        import os
        if (graph and len(jobs) > 1 and all(rg.graph is not None for rg in self._graphs)
                and os.environ.get("PDA_DP_THREADS", "1") != "0"):
            # one host thread per device: hipGraphLaunch of a ~500-node step costs ~2 ms of host
            # time, and CUDAGraph.replay releases the GIL, so N replicas enqueue concurrently
            # instead of staggering device i's start by i x 2 ms (captures stay on this thread)
            streams = [torch.cuda.current_stream(rg.dev) for rg in self._graphs]
            list(self._pool().map(lambda j: j[0][0].run(j[0][1], j[0][2], True, j[1]),
                                  zip(jobs, streams)))
        else:
            for rg, x, y in jobs:
                rg.run(x, y, graph)
        if self.replicas:
            self._reduce_grads()
        else:
            self.module._grads_zero = False
        optimizer.step()
        dev0 = torch.device("cuda", self.output_device)
        loss = torch.zeros((), dtype=torch.float32, device=dev0)
        for rg, x in zip(self._graphs, xs):
            loss += rg.loss.to(dev0, non_blocking=True) * (x.shape[0] / B)
        return loss

    def _pool(self):
        if getattr(self, "_executor", None) is None:
            from concurrent.futures import ThreadPoolExecutor
            self._executor = ThreadPoolExecutor(max_workers=len(self.device_ids),
                                                thread_name_prefix="dp-replay")
        return self._executor

    def _arm_callback(self, g):
        if not self._armed:
            self._armed = True
            torch.autograd.Variable._execution_engine.queue_callback(self._reduce_grads)
        return g


class _ReplicaGraph:
    """forward + CE loss/gradient + backward of one native replica, captured in a HIP graph on
    the replica's device; inputs are copied into static buffers before each replay."""

    def __init__(self, m, shape, global_batch: int) -> None:
        self.m = m
        self.dev = m.device
        self.gscale = 1.0 / global_batch
        with torch.cuda.device(self.dev):
            self.x = torch.empty(shape, dtype=m.dtype, device=self.dev)
            self.y = torch.empty(shape[0], dtype=torch.int64, device=self.dev)
        self.graph = None
        self.loss = None

    def _body(self) -> None:
        from ..ops import native_ops as K
        m = self.m
        B = self.x.shape[0]
        logits = m.native_forward(self.x, train=True, save=True)
        loss = torch.empty((), dtype=torch.float32, device=self.dev)
        rows = torch.empty(B, dtype=torch.float32, device=self.dev)
        dlog16 = torch.empty(B, m.fc_rows, dtype=m.dtype, device=self.dev)
        K.xent(logits, self.y, rows, loss, dlog=dlog16, gscale=self.gscale)
        m._grads_zero = True          # every step overwrites the flat gradient
        m.native_backward(dlog16)
        self.loss = loss

    def run(self, x: torch.Tensor, y: torch.Tensor, graph: bool = True,
            stream: Optional[torch.cuda.Stream] = None) -> None:
        """``stream``: the caller's current stream on this device. A worker thread's current
        stream is its own (the default stream), so a replay issued from the DataParallel thread
        pool runs on the caller's stream explicitly and stays ordered with the input production
        before it and the gradient reduction / optimizer step after it."""
        with torch.cuda.device(self.dev), torch.cuda.stream(stream or torch.cuda.current_stream(self.dev)):
            self.x.copy_(x, non_blocking=True)
            self.y.copy_(y, non_blocking=True)
            if not graph:                  # same schedule, launched eagerly (tests / debugging)
                self._body()
                return
            if self.graph is not None:
                self.graph.replay()
                self.loss = self._graph_loss
                return
            cur = torch.cuda.current_stream(self.dev)
            side = torch.cuda.Stream(self.dev)
            side.wait_stream(cur)
            with self.m.graph_schedule():
                with torch.cuda.stream(side):
                    self._body()               # the real step for this batch (also sizes workspaces)
                cur.wait_stream(side)
                eager = self.loss
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    self._body()
            self.graph = g
            self._graph_loss, self.loss = self.loss, eager
