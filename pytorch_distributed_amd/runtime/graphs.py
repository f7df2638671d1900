"""HIP-graph capture of one full native training step.

The reference's step is ~500 autograd-recorded ATen/cuDNN launches issued from Python every
iteration. The native engine already collapses the network into one explicit
schedule of our gfx950 kernels (``models/native.py``); this module goes one step further and
records that whole schedule -- on-device batch generation, forward, fused loss+gradient,
backward (main stream + the weight-gradient stream, forked and joined with events), fused SGD,
AMP loss-scale update -- into ONE HIP graph, replayed with a single launch per step:

* the host cost per step drops from ~600 kernel launches (ctypes + allocator + Python) to one
  ``hipGraphLaunch`` plus a 1-element fill (the batch's first sample id); this is what keeps a
  single-process multi-GPU driver (DataParallel) and small per-GPU batches from being
  launch-bound, and removes inter-launch gaps on the device;
* every buffer the step touches has a fixed address (workspaces are grown by the eager step
  that precedes capture; activations come from the graph's private memory pool);
* values that change between steps are device-resident (sample-id offset, AMP loss scale, found-inf
  flag) -- the only host-side hyper-parameter baked into the graph, the learning rate, triggers
  a re-capture when the LR scheduler changes it.

Used by :class:`~pytorch_distributed_amd.models.native.NativeTrainer` (``bench.py --graph``) and the
single-GPU entrypoint's training loop (``MX_GRAPH=1``, :mod:`pytorch_distributed_amd.trainer`).
"""
from __future__ import annotations

import os
from typing import Callable, Optional

import torch

from ..ops import native_ops as K

__all__ = ["GraphedNativeStep", "native_train_step", "single_queue_graphs",
           "request_single_queue_graphs"]


def native_train_step(model, opt, x: torch.Tensor, y: torch.Tensor, scaler=None) -> torch.Tensor:
    """forward -> CE loss + d(loss)/d(logits) in one kernel -> native backward -> fused SGD, with no
    autograd bookkeeping (the same kernel sequence as ``loss.backward(); opt.step()`` through the
    module's autograd node). Returns the (unscaled) mean loss as a device scalar."""
    B = x.shape[0]
    logits = model.native_forward(x, train=True, save=True)
    loss = torch.empty((), dtype=torch.float32, device=logits.device)
    rows = torch.empty(B, dtype=torch.float32, device=logits.device)
    dlog16 = torch.empty(B, model.fc_rows, dtype=model.dtype, device=logits.device)
    gdev = None
    if scaler is not None and scaler.enabled:
        scaler._lazy_init(logits.device)
        gdev = scaler.scale_tensor          # d(scale * loss) / d(loss), device-resident
    K.xent(logits, y, rows, loss, dlog=dlog16, gscale=1.0 / B, gdev=gdev)
    model.native_backward(dlog16)
    if gdev is not None:
        # inf check + scale update (one kernel), unscale + skip-on-overflow inside the fused SGD
        opt.step_amp(scaler.scale_tensor, scaler.found_inf, scaler._growth_tracker,
                     scaler.growth_factor, scaler.backoff_factor, scaler.growth_interval)
    else:
        opt.step()
    opt.zero_grad()
    return loss


# HIP graph launch queues. By default the HIP runtime spreads a graph's independent branches over
# internal streams; DEBUG_HIP_FORCE_GRAPH_QUEUES=1 launches every graph on one queue. A full GPU test
# session once segfaulted inside hipGraphLaunch (an out-of-range read of a per-graph stream list in
# libamdhip64.so) on the DataParallel replica graphs after ~85 tests, and =1 removed it
# (profiles/ab_r4.md section 7). Round 5 (profiles/ab_r5.md section 7, tools/graph_queue_repro.py):
# * the "immediate core dump under =0" of round 4 was the degenerate ZERO-queue setting -- =0
#   crashes (SIGFPE) inside capture_end for ANY captured graph, even a linear one without a fork;
#   it is not HIP's default;
# * under the real default (variable unset) the standalone reproducer (fork/join captures, segment
#   graphs sharing a pool, side graphs, up to 4 replica threads x 16 graphs x 500 replays) and the
#   DataParallel replica graphs (tests/test_dp_gpu.py, 40 steps bit-exact vs eager) run clean; the
#   long-session crash was not reproduced standalone.
# The variable is read ONCE, when HIP initialises: the entry points that replay graphs request
# single-queue launch before their first HIP call (resnet_dp.py, `bench.py --dp / --graph 1`, the
# GPU test session), and the graph paths replay only under it (else eager launches + a warning) --
# the configuration that ran every long session clean.
GRAPH_QUEUES_VAR = "DEBUG_HIP_FORCE_GRAPH_QUEUES"


def hip_runtime_started() -> bool:
    """Whether the HIP/HSA runtime of this process has initialised -- it then holds ``/dev/kfd``
    open. ``torch.cuda.is_initialized()`` alone misses it: ``device_count()`` / ``is_available()``
    start the runtime (which reads GRAPH_QUEUES_VAR once) without setting torch's flag."""
    if torch.cuda.is_initialized():
        return True
    try:
        for fd in os.listdir("/proc/self/fd"):
            try:
                if os.readlink(f"/proc/self/fd/{fd}") == "/dev/kfd":
                    return True
            except OSError:
                continue
    except OSError:
        pass
    return False


# the variable's value as last observed while the runtime had NOT started (the value it reads at
# its start unless changed in between); at module import, and again at every query made before
# the runtime starts. A module imported after the runtime started keeps the import-time value.
_QUEUES_SEEN = os.environ.get(GRAPH_QUEUES_VAR)


def single_queue_graphs() -> bool:
    """Whether HIP graphs launch on one queue in this process (see GRAPH_QUEUES_VAR): the variable
    must have been "1" before the HIP runtime started. A value set after the runtime started (by
    then it has read the variable) is not trusted."""
    global _QUEUES_SEEN
    if not hip_runtime_started():
        _QUEUES_SEEN = os.environ.get(GRAPH_QUEUES_VAR)
    return _QUEUES_SEEN == "1"


def request_single_queue_graphs() -> bool:
    """Ask for single-queue graph launch if HIP has not started yet in this process (an explicit
    setting is kept); returns whether graph replay is safe here (:func:`single_queue_graphs`)."""
    if not hip_runtime_started() and os.environ.get(GRAPH_QUEUES_VAR) is None:
        os.environ[GRAPH_QUEUES_VAR] = "1"
    return single_queue_graphs()


_WARNED = set()


def graphs_unsafe_warning(what: str) -> None:
    if what in _WARNED:
        return
    _WARNED.add(what)
    import warnings
    warnings.warn(f"{what}: HIP graph replay disabled -- {GRAPH_QUEUES_VAR}=1 was not set before "
                  "HIP started (the runtime's multi-queue graph launch crashes on these graphs); "
                  "launching eagerly", RuntimeWarning)


class GraphedNativeStep:
    """Capture-once / replay-per-step driver of :func:`native_train_step`.

    ``gen(ids) -> (x, y)`` is the on-device batch generator; the batch's sample ids are
    ``first_id + arange(batch)`` with ``first_id`` held in a device scalar, so one graph serves
    every step. The first :meth:`run` executes the step eagerly (on a side stream, which also
    grows every workspace to its final size) and then captures it; later calls replay.
    """

    def __init__(self, model, opt, gen: Callable, batch: int, scaler=None,
                 device: Optional[torch.device] = None) -> None:
        self.model, self.opt, self.gen, self.batch, self.scaler = model, opt, gen, batch, scaler
        self.device = torch.device(device) if device is not None else model.device
        self.ids_base = torch.arange(batch, dtype=torch.int64, device=self.device)
        self.ids_off = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.loss: Optional[torch.Tensor] = None
        self._lr = None
        self.captures = 0

    def _body(self) -> None:
        if self.gen is None:      # inputs from the caller: static buffers filled by run_batch
            x, y = self._sx, self._sy
        else:
            x, y = self.gen(self.ids_base + self.ids_off)
        self.loss = native_train_step(self.model, self.opt, x, y, self.scaler)

    def accepts(self, x: torch.Tensor) -> bool:
        """Whether :meth:`run_batch` can replay this batch (its shape is the captured one)."""
        return getattr(self, "_sx", None) is None or tuple(x.shape) == tuple(self._sx.shape)

    def run_batch(self, x: torch.Tensor, y: torch.Tensor) -> None:
        """One step on a caller-provided batch (``gen=None``): copied into static buffers that the
        graph reads, then replayed (captured on the first call / after an LR change)."""
        if getattr(self, "_sx", None) is None:
            self._sx = torch.empty_like(x, device=self.device)
            self._sy = torch.empty_like(y, device=self.device)
        self._sx.copy_(x, non_blocking=True)
        self._sy.copy_(y, non_blocking=True)
        self.run(None)

    def run(self, first_id: Optional[int]) -> None:
        if first_id is not None:
            self.ids_off.fill_(int(first_id))
        lr = self.opt.param_groups[0]["lr"]
        if self.graph is not None and lr == self._lr:
            self.graph.replay()
            self.loss = self._graph_loss
            return
        # eager step (the real step for this batch), off the default stream as graph capture
        # requires, then record the identical schedule
        cur = torch.cuda.current_stream(self.device)
        side = torch.cuda.Stream(self.device)
        side.wait_stream(cur)
        with self.model.graph_schedule():
            with torch.cuda.stream(side):
                self._body()
            cur.wait_stream(side)
            eager_loss = self.loss
            self.graph = None
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._body()
        self.graph = g
        self._graph_loss = self.loss      # written by each replay
        self.loss = eager_loss            # this step's value (the capture executed nothing)
        self._lr = lr
        self.captures += 1
