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
* the flat gradients are SUM-all-reduced across the local GPUs by grouped
  in-process RCCL collectives (``ncclCommInitAll`` communicator,
  :class:`~pytorch_distributed_amd.parallel.rccl.RcclGroup`) -- with the
  graph-replayed step, one per stage slice of the flat gradient on per-device
  comm streams, overlapped with the replay of the next backward segment
  (``PDA_DP_SEGMENTS``) -- and every replica runs the fused SGD itself
  (replicated update: mathematically identical to reduce-to-GPU0 + step +
  broadcast, with no per-step weight broadcast);
* BN buffers (213 KB) are broadcast from replica 0 before each training forward,
  which is what torch's per-step ``replicate`` achieves for them.

For arbitrary (non-native) modules it falls back to persistent deep-copied
replicas with a parameter refresh before each forward and a gradient
reduction into replica 0 after backward -- the same math as ``nn.DataParallel``.
"""
from __future__ import annotations

import contextlib
import copy
import os
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
        # HIP events at the end of backward and after the last gradient all-reduce of the next
        # graph-replayed step (exposed_comm_ms); diagnostics only
        self.timing = False
        # one device: replay the replica graphs anyway (bench.py dp_replay_ms_per_step)
        self.force_replay = os.environ.get("PDA_DP_FORCE_REPLAY", "0") == "1"
        # host-side bound on one reduce interval's replay enqueue per device worker (its segments'
        # graph launches, ~ms): a worker that raises or never returns becomes an exception in the
        # caller
        self.replay_timeout_s = float(os.environ.get("PDA_DP_REPLAY_TIMEOUT_S", "120"))
        self._ev_bwd = self._ev_comm = None

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
    def _reduce_slice(self, lo: int, hi: int, streams=None) -> None:
        """SUM-all-reduce ``flat_grad[lo:hi]`` over the replicas, on ``streams`` (one per replica;
        default: the devices' current streams)."""
        ts = [m.flat_grad[lo:hi] for m in self.all_modules]
        if self.group is not None:
            self.group.all_reduce(ts, streams=streams)
            return
        # replicas sharing a device (tests): plain copies, on replica 0's stream, ordered after every
        # replica's stream (each waited only on its own replica's work) and before all of them
        if streams is not None:
            for c in streams[1:]:
                streams[0].wait_stream(c)
        ctx = torch.cuda.stream(streams[0]) if streams is not None else contextlib.nullcontext()
        with ctx:
            total = ts[0].clone()
            for t in ts[1:]:
                total.add_(t.to(total.device))
            for t in ts:
                t.copy_(total, non_blocking=True)
        if streams is not None:
            for c in streams[1:]:
                c.wait_stream(streams[0])

    @torch.no_grad()
    def _reduce_grads(self) -> None:
        self._armed = False
        if self._native:
            self._reduce_slice(0, self.module.numel)
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
        ok = (self._native and bool(self.device_ids) and (scaler is None or not scaler.enabled)
              and os.environ.get("MX_GRAPH", "1") != "0")
        if ok:
            from ..runtime.graphs import graphs_unsafe_warning, single_queue_graphs
            if not single_queue_graphs():   # replica graphs need the single-queue graph launch
                graphs_unsafe_warning("DataParallel")
                return False
        return ok

    def train_step(self, samples: torch.Tensor, labels: torch.Tensor, optimizer,
                   graph: bool = True) -> torch.Tensor:
        """One DP training step with every replica's forward + loss + backward replayed from a HIP
        graph: ONE host launch per device instead of ~600 (the eager schedule costs ~8 ms of host
        time per device per ResNet-50 step, so one thread driving 8 GPUs eagerly would be
        launch-bound; see ``tools/host_overhead.py``). Same math as ``crit(dp(x), y).backward();
        optimizer.step()``: the loss is the mean over the GLOBAL batch (each replica's gradient
        is scaled by 1/B_global), BN statistics are per replica, BN buffers follow replica 0,
        gradients are SUM-all-reduced by grouped RCCL calls (one per stage slice, overlapped with
        the rest of the backward: :meth:`_replay_overlapped`), then the replicated fused SGD."""
        xs = torch.chunk(samples, len(self.device_ids), 0)
        ys = torch.chunk(labels, len(self.device_ids), 0)
        return self.train_step_chunks(xs, ys, optimizer, graph)

    def train_step_chunks(self, xs, ys, optimizer, graph: bool = True) -> torch.Tensor:
        """:meth:`train_step` on per-replica input chunks (e.g. generated on each GPU directly,
        skipping the scatter from ``device_ids[0]``)."""
        if graph and not self.replicas and not self.force_replay:
            # one device: the module's own (eager, two-stream) step, as torch's DataParallel calls
            # the module directly for a single device; replay only pays where one host thread
            # drives several GPUs. ``force_replay`` keeps the replica graphs on one device, so the
            # path an N > 1 run takes is measurable on one (bench.py dp_replay_ms_per_step)
            graph = False
        if graph:
            from ..runtime.graphs import graphs_unsafe_warning, single_queue_graphs
            if not single_queue_graphs():   # the replica graphs need the single-queue launch
                graphs_unsafe_warning("DataParallel")
                graph = False
        self._broadcast_state()
        B = sum(x.shape[0] for x in xs)
        if getattr(self, "_graphs", None) is None or [x.shape for x in xs] != self._graph_shapes:
            splits = self._segment_bounds()
            self._graphs = [_ReplicaGraph(m, x.shape, B, splits) for m, x in zip(self.all_modules, xs)]
            self._graph_shapes = [x.shape for x in xs]
        jobs = list(zip(self._graphs, xs, ys))
        streams = [torch.cuda.current_stream(rg.dev) for rg in self._graphs]
        replay = graph and all(rg.graphs for rg in self._graphs)
        if replay and self.replicas:
            self._replay_overlapped(jobs, streams)
            if len(jobs[0][0].graphs) > 1 and not getattr(self, "_segments_verified", False):
                self._verify_segmented_reduce(optimizer)
                loss = self._step_loss(xs, B)   # this step's graphs hold its losses
                if getattr(self, "_force_single_segment", False):
                    self._graphs = None         # re-captured without split points next step
                return loss
        else:
            for rg, x, y in jobs:
                rg.run(x, y, graph)
            if self.replicas:
                self._reduce_grads()
            else:
                self.module._grads_zero = False
        optimizer.step()
        return self._step_loss(xs, B)

    def _step_loss(self, xs, B: int) -> torch.Tensor:
        dev0 = torch.device("cuda", self.output_device)
        loss = torch.zeros((), dtype=torch.float32, device=dev0)
        for rg, x in zip(self._graphs, xs):
            loss += rg.loss.to(dev0, non_blocking=True) * (x.shape[0] / B)
        return loss

    @torch.no_grad()
    def _verify_segmented_reduce(self, optimizer) -> None:
        """First segmented step of a DataParallel: every replica must now hold the SAME summed flat
        gradient (bit-exact; each slice went through one grouped all-reduce). On a mismatch -- a
        slice that was never reduced, or reduced out of order -- the per-stage overlap is turned off
        (``PDA_DP_SEGMENTS=0`` behaviour: one graph, one all-reduce after backward), this step's
        update is taken from replica 0 (its state is copied to every replica after the step), and a
        warning says so: training continues consistent instead of silently diverging."""
        from ..bench_step import tensor_checksum
        for d in self.device_ids:
            torch.cuda.synchronize(d)
        sums = [tensor_checksum([m.flat_grad]).cpu() for m in self.all_modules]
        ok = all(torch.equal(sums[0], c) for c in sums[1:])
        optimizer.step()
        self._segments_verified = True
        if ok:
            return
        import warnings
        warnings.warn("DataParallel: the per-stage gradient all-reduce left replicas with different "
                      "gradients; falling back to one all-reduce after backward (PDA_DP_SEGMENTS=0) "
                      "and re-syncing every replica from replica 0", RuntimeWarning)
        self._force_single_segment = True   # (train_step_chunks drops the graphs after the loss)
        m0 = self.module
        opt0 = optimizer.opts[0] if hasattr(optimizer, "opts") else None
        for i, r in enumerate(self.replicas):
            with torch.cuda.device(r.device):
                r.flat_params.copy_(m0.flat_params)
                r.flat_bufstore.copy_(m0.flat_bufstore)
                if opt0 is not None:
                    optimizer.opts[i + 1].flat_mom.copy_(opt0.flat_mom)
                r.refresh_shadow()
        for d in self.device_ids:
            torch.cuda.synchronize(d)

    def _segment_bounds(self) -> List[int]:
        """Where each replica graph is split (``PDA_DP_SEGMENTS``): "stage" (default) after the
        backward of layer4, layer3 and layer2 -- the fc+layer4 slice (~68 MB of the 102 MB f32
        gradient of ResNet-50) is all-reduced while layer3..1 run backward, the exposed tail is
        the ~1 MB layer1+stem slice; "0": one graph, one all-reduce after backward."""
        mode = os.environ.get("PDA_DP_SEGMENTS", "stage")
        if mode not in ("stage", "0"):
            raise ValueError(f"PDA_DP_SEGMENTS={mode!r}: expected stage or 0")
        if (mode == "0" or getattr(self, "_force_single_segment", False) or not self.replicas
                or not hasattr(self.module, "stage_bounds")):
            return []
        return self.module.stage_bounds()

    def _comm_streams(self):
        if getattr(self, "_cstreams", None) is None:
            self._cstreams = [torch.cuda.Stream(torch.device("cuda", d)) for d in self.device_ids]
        return self._cstreams

    def _replay_overlapped(self, jobs, streams) -> None:
        """Replay segment s of every replica (its main-chain graph on the replica's stream and, in
        side-split captures, its weight-gradient graph on the replica's second stream), and after
        each segment that completes a gradient slice all-reduce that slice on per-device comm
        streams -- ordered after both streams of every replica -- while the next segments replay;
        the replicas' streams join the comm and second streams before the optimizer step.
        ``self.timing``: HIP events at the end of backward and after the last all-reduce
        (``exposed_comm_ms``)."""
        cs = self._comm_streams()
        rg0 = jobs[0][0]
        nseg = len(rg0.graphs)
        ends = rg0.seg_reduce
        # (replicas that share a device replay from this thread: concurrent hipGraphLaunch calls
        # onto ONE device from two host threads crashed inside the HIP runtime in a long GPU test
        # session -- a segfault in CUDAGraph.replay; distinct devices keep one thread each)
        threaded = (len(jobs) > 1 and os.environ.get("PDA_DP_THREADS", "1") != "0"
                    and len(set(self.device_ids)) == len(self.device_ids))
        timing = self.timing
        lo = 0
        s = 0
        while s < nseg:
            # the segments up to the next all-reduce point (or the last): with a side graph per
            # weight gradient a step has ~65 segments but only 4 reduce points, and one worker task
            # per device per reduce interval keeps the host's per-segment dispatch cost out of the
            # N-device enqueue
            e = s
            while e < nseg - 1 and ends[e] is None:
                e += 1
            if threaded:
                # one host thread per device: hipGraphLaunch of a segment costs host time and
                # CUDAGraph.replay releases the GIL, so the N replicas enqueue concurrently instead
                # of staggering device i's start by i launches
                run_workers(self._pool(), [
                    (lambda a=a, s0=s, s1=e: a[0][0].replay_range(s0, s1, a[0][1], a[0][2], a[1]))
                    for a in zip(jobs, streams)], self.replay_timeout_s,
                    [f"cuda:{rg.dev.index}" for rg, _, _ in jobs])
            else:
                for k in range(s, e + 1):
                    for (rg, x, y), st in zip(jobs, streams):
                        rg.replay(k, x, y, st)
            if timing and e == nseg - 1:
                self._ev_bwd = [torch.cuda.Event(enable_timing=True) for _ in streams]
                for ev, st, (rg, _, _) in zip(self._ev_bwd, streams, jobs):
                    rg.join_side(st)
                    ev.record(st)
            hi = ends[e]
            s = e + 1
            if hi is None:
                continue
            for c, st, (rg, _, _) in zip(cs, streams, jobs):
                c.wait_stream(st)
                if rg.side_split:
                    c.wait_stream(rg.m._side)
            self._reduce_slice(lo, hi, streams=cs)
            lo = hi
        if timing:
            self._ev_comm = [torch.cuda.Event(enable_timing=True) for _ in cs]
            for e, c in zip(self._ev_comm, cs):
                e.record(c)
        for c, st, (rg, _, _) in zip(cs, streams, jobs):
            rg.join_side(st)
            st.wait_stream(c)
        for m in self.all_modules:
            m._grads_zero = False

    def exposed_comm_ms(self) -> Optional[float]:
        """After a step with ``timing = True`` has completed: max over devices of (last gradient
        all-reduce done - backward done)."""
        if self._ev_comm is None:
            return None
        return max(b.elapsed_time(c) for b, c in zip(self._ev_bwd, self._ev_comm))

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


def run_workers(pool, fns, timeout_s: float, names=None) -> list:
    """Run ``fns`` on the executor ``pool`` and wait at most ``timeout_s`` seconds for all of them:
    the first worker exception is re-raised here (naming its device), and workers still running at
    the deadline raise TimeoutError instead of hanging the step. Results in ``fns`` order."""
    from concurrent.futures import FIRST_EXCEPTION, wait
    names = names or [str(i) for i in range(len(fns))]
    futs = [pool.submit(f) for f in fns]
    done, pending = wait(futs, timeout=timeout_s, return_when=FIRST_EXCEPTION)
    for f, n in zip(futs, names):
        if f in done and f.exception() is not None:
            for p in pending:
                p.cancel()
            raise RuntimeError(f"DataParallel replay worker for {n} failed: "
                               f"{type(f.exception()).__name__}: {f.exception()}") from f.exception()
    if pending:
        late = [n for f, n in zip(futs, names) if f in pending]
        raise TimeoutError(f"DataParallel replay worker(s) for {late} did not return within "
                           f"{timeout_s:.0f} s")
    return [f.result() for f in futs]


class _ReplicaGraph:
    """forward + CE loss/gradient + backward of one native replica, captured as HIP graphs on the
    replica's device; inputs are copied into static buffers before each replay.

    ``splits`` (flat-gradient offsets, ``NativeResNet.stage_bounds``): where DataParallel
    all-reduces a completed gradient slice between segment replays.

    ``side_split`` (``PDA_DP_SIDE=1``, default): the weight-gradient kernels are recorded in graphs
    of their own. The HIP runtime replays one captured graph's fork/join DAG almost serially
    (``profiles/rocprof_r3_graph_replay.md``: 368 of ~410 kernels on one queue), which loses the
    two-stream overlap of the eager step; so the capture ends a main-chain graph after every
    residual block's backward and records the weight gradients queued during that block as a
    second graph, replayed on the replica's second stream after the main segment -- it runs beside
    the next block's data-gradient chain, as the eager schedule's "block" fork granularity does.
    Without it, a segment ends only at the split offsets, after joining the weight-gradient stream."""

    def __init__(self, m, shape, global_batch: int, splits: Sequence[int] = ()) -> None:
        self.m = m
        self.dev = m.device
        self.gscale = 1.0 / global_batch
        self.splits = list(splits)
        side = os.environ.get("PDA_DP_SIDE", "conv")
        if side not in ("conv", "1", "0"):
            raise ValueError(f"PDA_DP_SIDE={side!r}: expected conv, 1 or 0")
        self.side_split = getattr(m, "_side", None) is not None and side != "0"
        # "conv": a side graph per weight gradient (the main segment ends where its inputs are
        # complete, so it starts as early as in the eager schedule); "1": one per residual block
        self.side_per_conv = self.side_split and side == "conv"
        self._fork_ev = None   # main -> side hand-off event of the replay (native_ops.fork_event_create)
        with torch.cuda.device(self.dev):
            self.x = torch.empty(shape, dtype=m.dtype, device=self.dev)
            self.y = torch.empty(shape[0], dtype=torch.int64, device=self.dev)
        self.graphs: List[torch.cuda.CUDAGraph] = []     # main-chain segments
        self.sides: List[Optional[torch.cuda.CUDAGraph]] = []   # weight-gradient graph per segment
        self.seg_reduce: List[Optional[int]] = []        # slice end all-reducible after segment s
        self.loss = None
        self._capturing = False
        self._pool_h = None

    @property
    def graph(self):
        return self.graphs[0] if self.graphs else None

    def _capture_side(self):
        """Record the queued weight-gradient kernels as one graph on the second stream."""
        m = self.m
        if not m._wbatch:
            return None
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(m._side):
            g.capture_begin(pool=self._pool_h)
            try:
                for fn in m._wbatch:
                    fn(m.ws_w)
            finally:
                g.capture_end()
        m._wbatch.clear()
        return g

    def _end_segment(self, upto: Optional[int]) -> None:
        self.graphs[-1].capture_end()
        if self._pool_h is None:   # (torch hands out the pool id only after a finished capture)
            self._pool_h = self.graphs[0].pool()
        self.sides.append(self._capture_side() if self.side_split else None)
        self.seg_reduce.append(upto)

    def _split_conv(self) -> None:
        """NativeResNet.wgrad_hook (side_per_conv): end the main segment after the work a weight
        gradient just queued depends on and record that weight gradient as a side graph."""
        if not self._capturing:
            return
        # (second-stream work forked inside the segment -- the shortcut branch's data gradient --
        # joins it: a capture cannot end with an unjoined fork)
        torch.cuda.current_stream(self.dev).wait_stream(self.m._side)
        self._end_segment(None)
        g = torch.cuda.CUDAGraph()
        g.capture_begin(pool=self._pool_h)
        self.graphs.append(g)

    def _split(self, upto: int) -> None:
        """NativeResNet.segment_hook, after each residual block's backward."""
        if self.side_split and self._capturing:
            if self.side_per_conv and upto not in self.splits:
                return   # every weight gradient already ended a segment: no block boundary needed
            self._end_segment(upto if upto in self.splits else None)
            g = torch.cuda.CUDAGraph()
            g.capture_begin(pool=self._pool_h)
            self.graphs.append(g)
            return
        if upto not in self.splits:
            return
        # at a split offset join the weight-gradient stream (eager and captured schedules alike)
        # and, while capturing, start the next segment's graph
        self.m.join_side()
        if self._capturing:
            self._end_segment(upto)
            g = torch.cuda.CUDAGraph()
            g.capture_begin(pool=self._pool_h)
            self.graphs.append(g)

    def _body(self) -> None:
        from ..ops import native_ops as K
        m = self.m
        B = self.x.shape[0]
        # (set before the forward: conv mode also records the forward-time Gram work of the tail
        # folds as side graphs -- forked inside a segment graph, the runtime replayed it on the
        # main queue: ~0.8 ms/step of Gram / B-GEMM / reduce launches serialised into the chain)
        m.defer_side = self.side_split and self._capturing
        m.wgrad_hook = self._split_conv if self.side_per_conv else None
        try:
            logits = m.native_forward(self.x, train=True, save=True)
            loss = torch.empty((), dtype=torch.float32, device=self.dev)
            rows = torch.empty(B, dtype=torch.float32, device=self.dev)
            dlog16 = torch.empty(B, m.fc_rows, dtype=m.dtype, device=self.dev)
            K.xent(logits, self.y, rows, loss, dlog=dlog16, gscale=self.gscale)
            m._grads_zero = True          # every step overwrites the flat gradient
            m.segment_hook = self._split if (self.splits or self.side_split) else None
            m.native_backward(dlog16)
        finally:
            m.segment_hook = None
            m.defer_side = False
            m.wgrad_hook = None
        self.loss = loss

    def join_side(self, stream: torch.cuda.Stream) -> None:
        """Make ``stream`` wait for the replica's weight-gradient graphs replayed so far."""
        if self.side_split:
            stream.wait_stream(self.m._side)

    def replay(self, s: int, x: torch.Tensor, y: torch.Tensor,
               stream: Optional[torch.cuda.Stream] = None) -> None:
        """Replay segment ``s`` on ``stream`` (the caller's current stream on this device: a
        worker thread's own current stream is the default stream), then its weight-gradient graph
        on the second stream after it; segment 0 first takes the inputs."""
        self.replay_range(s, s, x, y, stream)

    def replay_range(self, s0: int, s1: int, x: torch.Tensor, y: torch.Tensor,
                     stream: Optional[torch.cuda.Stream] = None) -> None:
        """:meth:`replay` of segments ``s0 .. s1`` under one device context (host cost per segment:
        a main-graph launch, and for a side graph one event hand-off + its launch)."""
        with torch.cuda.device(self.dev):
            st = stream or torch.cuda.current_stream(self.dev)
            side_st = self.m._side
            for s in range(s0, s1 + 1):
                with torch.cuda.stream(st):
                    if s == 0:
                        self.x.copy_(x, non_blocking=True)
                        self.y.copy_(y, non_blocking=True)
                    self.graphs[s].replay()
                side = self.sides[s] if s < len(self.sides) else None
                if side is not None:
                    import ctypes as C
                    from ..ops import ext, native_ops as K
                    if self._fork_ev is None:
                        self._fork_ev = K.fork_event_create()
                    L = ext.lib()
                    K.check(L.pda_event_record(self._fork_ev, C.c_void_p(st.cuda_stream)),
                            "pda_event_record")
                    K.check(L.pda_stream_wait_event(C.c_void_p(side_st.cuda_stream), self._fork_ev),
                            "pda_stream_wait_event")
                    with torch.cuda.stream(side_st):
                        side.replay()
            self.loss = self._graph_loss

    def run(self, x: torch.Tensor, y: torch.Tensor, graph: bool = True,
            stream: Optional[torch.cuda.Stream] = None) -> None:
        """The whole step: eagerly (``graph=False``), by replaying every segment, or -- the first
        time -- eagerly for this batch and then captured for the next replays."""
        if graph and self.graphs:
            st = stream or torch.cuda.current_stream(self.dev)
            self.replay_range(0, len(self.graphs) - 1, x, y, st)
            self.join_side(st)
            return
        with torch.cuda.device(self.dev), torch.cuda.stream(stream or torch.cuda.current_stream(self.dev)):
            self.x.copy_(x, non_blocking=True)
            self.y.copy_(y, non_blocking=True)
            if not graph:                  # same schedule, launched eagerly (tests / debugging)
                self._body()
                return
            import gc
            cur = torch.cuda.current_stream(self.dev)
            side = torch.cuda.Stream(self.dev)
            side.wait_stream(cur)
            with self.m.graph_schedule(concurrent_side=self.side_split):
                with torch.cuda.stream(side):
                    self._body()               # the real step for this batch (also sizes workspaces)
                cur.wait_stream(side)
                eager = self.loss
                # what torch.cuda.graph does on entry, with capture_begin / capture_end by hand so
                # the backward can end one segment's graph and begin the next
                torch.cuda.synchronize(self.dev)
                gc.collect()
                torch.cuda.empty_cache()
                cap = torch.cuda.Stream(self.dev)
                cap.wait_stream(cur)
                if self.m._side is not None:
                    self.m._side.wait_stream(cur)
                with torch.cuda.stream(cap):
                    g = torch.cuda.CUDAGraph()
                    self.graphs, self.sides, self.seg_reduce = [g], [], []
                    self._capturing = True
                    ended = False
                    try:
                        self._pool_h = None
                        g.capture_begin()
                        self._body()
                        self._end_segment(self.m.numel)
                        ended = True
                        if self.side_split:
                            # tensors the weight-gradient graphs read stay allocated until every
                            # segment is recorded: a later segment must not reuse their memory
                            # while a side graph may still be reading it at replay
                            self.m._keep.clear()
                        want = sorted(self.splits) + [self.m.numel]
                        got = [u for u in self.seg_reduce if u is not None]
                        if got != want or len(self.sides) != len(self.graphs):
                            # a split offset the backward never reported: the gradient past it
                            # would never be all-reduced
                            raise RuntimeError(f"replica capture: all-reduce points {got}, "
                                               f"expected {want}")
                    except BaseException:
                        if not ended:   # leave no capture open on the stream
                            try:
                                self.graphs[-1].capture_end()
                            except Exception:   # noqa: BLE001 (already invalidated)
                                pass
                        self.graphs, self.sides, self.seg_reduce = [], [], []
                        raise
                    finally:
                        self._capturing = False
                cur.wait_stream(cap)
                if self.m._side is not None:
                    cur.wait_stream(self.m._side)
            self._graph_loss, self.loss = self.loss, eager
