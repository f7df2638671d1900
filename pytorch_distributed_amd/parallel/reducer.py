"""Gradient bucketing reducer (replacement for torch DDP's C++ ``Reducer``).

Reference behaviour relied upon: gradients are
averaged across ranks by bucketed all-reduces issued *during* backward, in
reverse parameter order, overlapping autograd.

Design (MI355X-first):

* every bucket is one contiguous flat buffer and each parameter's ``.grad`` is a
  *view* into it (``gradient_as_bucket_view``) -- no bucket copy-in/copy-out;
  with the native engine the whole model's gradients already live in ONE flat
  buffer laid out in gradient-production order, so buckets are just slices;
* bucket sizes are chosen for xGMI: middle buckets default to 32 MiB, the first
  (fc) bucket fires as soon as its gradient exists, and the *last* bucket (the one
  exposed after backward ends) is kept small (2 MiB) so the tail is short;
* xGMI cost model behind the defaults. An MI355X node is 8 GPUs, each with 7
  point-to-point xGMI links of ~153 GB/s. RCCL runs an 8-rank all-reduce over several channels
  so all 7 links carry traffic; each rank moves 2(n-1)/n * S bytes:

      T(S) ~= alpha + 2 * (7/8) * S / (7 * 153 GB/s * eta),  alpha ~ 15-30 us, eta ~ 0.6-0.8

  ResNet-50 has S_total = 102 MB of f32 gradients per step: ~0.25 ms of link time against
  ~20 ms of backward at bs 400, so bandwidth never binds. What the plan optimises instead:
    1. the number of collectives -- each costs alpha on the comm stream plus a kernel launch whose
       workgroups compete with backward for CUs. 32 MiB middle buckets give 5-6 collectives per
       step, and at 32 MiB alpha is < 10 % of T(S);
    2. the exposed tail -- the bucket completing when backward ends (stem + layer1) runs after the
       last backward kernel. Capping it at 2 MiB bounds the tail at ~alpha + 4 us (~30 us);
    3. alignment -- the native engine pads every bucket boundary to a multiple of
       8 ranks x 7 links x 256 B (``models/native.py`` BUCKET_QUANTUM), so RCCL's per-rank /
       per-channel chunks are equal and 256-B aligned for any world size dividing 8.
  ``bench.py`` reports the measured per-bucket all-reduce time and the exposed tail
  (``bucket_allreduce_ms``, ``exposed_comm_ms``) for N > 1, and ``xgmi_probe``: alpha, bus
  bandwidth and eta measured through the same communicator at 16 KiB-32 MiB, so the model's
  constants come from the node the driver runs;
* readiness: ``Tensor.register_post_accumulate_grad_hook`` (generic modules) or
  the native engine's ``on_grads_ready(offset)`` callback; a ready bucket is
  pre-scaled by 1/world and all-reduced (SUM) asynchronously through a
  :class:`~pytorch_distributed_amd.parallel.comm.Communicator` on its own HIP
  stream; the end-of-backward callback makes the compute stream wait for the
  outstanding collectives before the optimizer consumes the flat gradient.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from .comm import Communicator

__all__ = ["Bucket", "Reducer", "plan_buckets"]

MiB = 1 << 20


def plan_buckets(sizes_bytes: Sequence[int], cap_bytes: int, first_cap_bytes: int,
                 last_cap_bytes: Optional[int] = None) -> List[List[int]]:
    """Greedy grouping of consecutive items (already in gradient-production order).

    The first bucket is capped at ``first_cap_bytes`` (fires early, as torch's 1 MiB
    first bucket), middle buckets at ``cap_bytes``; optionally the trailing items are
    regrouped so the final bucket holds at most ``last_cap_bytes``.
    """
    out: List[List[int]] = []
    cur: List[int] = []
    cur_b = 0
    for i, b in enumerate(sizes_bytes):
        cap = first_cap_bytes if not out else cap_bytes
        if cur and cur_b + b > cap:
            out.append(cur)
            cur, cur_b = [], 0
        cur.append(i)
        cur_b += b
    if cur:
        out.append(cur)
    if last_cap_bytes is not None and len(out) >= 1:
        last = out[-1]
        tot = sum(sizes_bytes[i] for i in last)
        if tot > last_cap_bytes and len(last) > 1:
            # split the tail so the exposed final bucket is small
            tail: List[int] = []
            tb = 0
            for i in reversed(last):
                if tail and tb + sizes_bytes[i] > last_cap_bytes:
                    break
                tail.insert(0, i)
                tb += sizes_bytes[i]
            head = [i for i in last if i not in tail]
            out[-1:] = [head, tail] if head else [tail]
    return out


class Bucket:
    def __init__(self, index: int, buffer: torch.Tensor, params: List[torch.nn.Parameter],
                 offsets: List[int]) -> None:
        self.index = index
        self.buffer = buffer
        self.params = params
        self.offsets = offsets
        self.pending = len(params)
        self.got = set()      # indices of params whose gradient arrived this step
        self.work = None

    def view_for(self, j: int) -> torch.Tensor:
        p = self.params[j]
        return self.buffer[self.offsets[j]:self.offsets[j] + p.numel()].view_as(p)


class Reducer:
    """Generic per-parameter-hook reducer over arbitrary ``nn.Module`` parameters."""

    def __init__(self, params: Sequence[torch.nn.Parameter], comm: Communicator,
                 bucket_cap_mb: Optional[float] = None, first_bucket_mb: float = 1.0,
                 last_bucket_mb: Optional[float] = 2.0) -> None:
        self.comm = comm
        params = [p for p in params if p.requires_grad]
        order = list(reversed(params))  # reverse registration ~ gradient production order
        cap = int((bucket_cap_mb or 32.0) * MiB)
        groups = plan_buckets([p.numel() * p.element_size() for p in order], cap,
                              int(first_bucket_mb * MiB),
                              int(last_bucket_mb * MiB) if last_bucket_mb else None)
        self.buckets: List[Bucket] = []
        self._where = {}
        for bi, g in enumerate(groups):
            ps = [order[i] for i in g]
            dtype = ps[0].dtype
            numel = sum(p.numel() for p in ps)
            buf = torch.zeros(numel, dtype=dtype, device=ps[0].device)
            offs, o = [], 0
            for p in ps:
                offs.append(o)
                o += p.numel()
            b = Bucket(bi, buf, ps, offs)
            self.buckets.append(b)
            for j, p in enumerate(ps):
                self._where[id(p)] = (b, j)
                p.grad = b.view_for(j)
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in params]
        self._armed = False
        self.enabled = True

    @property
    def bucket_bytes(self) -> List[int]:
        return [b.buffer.numel() * b.buffer.element_size() for b in self.buckets]

    # -- backward-time machinery ---------------------------------------------------------
    def _arm(self) -> None:
        if self._armed:
            return
        self._armed = True
        for b in self.buckets:
            b.pending = len(b.params)
            b.got = set()
            b.work = None
        torch.autograd.Variable._execution_engine.queue_callback(self._finalize)

    def _on_grad(self, p: torch.nn.Parameter) -> None:
        if not self.enabled:
            return
        self._arm()
        b, j = self._where[id(p)]
        view = b.view_for(j)
        if p.grad is None:
            view.zero_()
        elif p.grad.data_ptr() != view.data_ptr():
            view.copy_(p.grad)
        p.grad = view
        b.got.add(j)
        b.pending -= 1
        if b.pending == 0:
            self._launch(b)

    def _launch(self, b: Bucket) -> None:
        b.buffer.div_(self.comm.world_size)
        b.work = self.comm.all_reduce_async(b.buffer)

    def _finalize(self) -> None:
        for b in self.buckets:
            if b.work is None:
                # params that received no gradient this step contribute ZEROS (their bucket view
                # still holds last step's values: never reduce those)
                for j, p in enumerate(b.params):
                    if j not in b.got:
                        b.view_for(j).zero_()
                    if p.grad is None or p.grad.data_ptr() != b.view_for(j).data_ptr():
                        p.grad = b.view_for(j)
                self._launch(b)
        for b in self.buckets:
            self.comm.wait(b.work)
            b.work = None
        self._armed = False

    def remove(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
