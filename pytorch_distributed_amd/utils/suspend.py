"""Preemption ("suspend") protocol: native replacement for ``hfai.client``.

The reference polls ``hfai.client.receive_suspend_command()`` every step and,
when the cluster scheduler asks, saves ``latest.pt`` and calls
``hfai.client.go_suspend()`` (reference ``restnet_ddp.py:35-47``).
Here a suspend request is either

* a signal (``SIGUSR1`` by default; ``SIGTERM`` optionally), or
* a sentinel file (``MX_SUSPEND_FILE``; its existence means "suspend"), or
* a step trigger ``MX_SUSPEND_AT_STEP=<global step>`` (fault-injection in tests).

In DDP the decision is made collectively (MAX all-reduce of the local flag) so
every rank checkpoints/exits at the same step -- fixing quirk Q5, where only
rank 0 polled and the other ranks ran on into collectives.
``go_suspend()`` exits the process with :data:`REQUEUE_EXIT_CODE` so a job
scheduler can re-queue; rerunning the same command resumes from ``latest.pt``.
"""
from __future__ import annotations

import os
import signal
import sys
import threading
from typing import Optional

__all__ = ["SuspendMonitor", "REQUEUE_EXIT_CODE", "receive_suspend_command", "go_suspend"]

REQUEUE_EXIT_CODE = 75  # EX_TEMPFAIL


class SuspendMonitor:
    def __init__(self, signals=(signal.SIGUSR1,), sentinel: Optional[str] = None,
                 at_step: Optional[int] = None) -> None:
        self._flag = threading.Event()
        self.sentinel = sentinel if sentinel is not None else os.environ.get("MX_SUSPEND_FILE")
        env_step = os.environ.get("MX_SUSPEND_AT_STEP")
        self.at_step = at_step if at_step is not None else (int(env_step) if env_step else None)
        self.global_step = 0
        self._installed = []
        if threading.current_thread() is threading.main_thread():
            for s in signals:
                try:
                    prev = signal.signal(s, self._on_signal)
                    self._installed.append((s, prev))
                except (ValueError, OSError):
                    pass

    def _on_signal(self, signum, frame) -> None:  # pragma: no cover - exercised via subprocess
        self._flag.set()

    def request(self) -> None:
        self._flag.set()

    def tick(self) -> None:
        self.global_step += 1

    def local_requested(self) -> bool:
        if self._flag.is_set():
            return True
        if self.sentinel and os.path.exists(self.sentinel):
            return True
        if self.at_step is not None and self.global_step >= self.at_step:
            return True
        return False

    def requested(self, group=None) -> bool:
        """Collective decision: True on every rank iff any rank was asked to suspend.

        The collective runs every ``MX_SUSPEND_POLL`` steps (default 1, the reference polls every
        step); all ranks tick in lockstep, so they agree on which steps poll."""
        local = self.local_requested()
        import torch.distributed as dist
        every = max(1, int(os.environ.get("MX_SUSPEND_POLL", "1")))
        if self.global_step % every:
            return False
        if dist.is_available() and dist.is_initialized():
            import torch
            from ..launch import host_group
            # a host value: all-reduced on the gloo host group (no device collective, no stall of
            # the compute stream)
            t = torch.tensor([1.0 if local else 0.0])
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group if group is not None else host_group())
            return bool(t.item() > 0)
        return local

    def restore(self) -> None:
        for s, prev in self._installed:
            signal.signal(s, prev)
        self._installed = []


_default: Optional[SuspendMonitor] = None


def _monitor() -> SuspendMonitor:
    global _default
    if _default is None:
        _default = SuspendMonitor()
    return _default


def receive_suspend_command() -> bool:
    """Drop-in for ``hfai.client.receive_suspend_command()`` (local decision)."""
    return _monitor().local_requested()


def go_suspend(code: int = REQUEUE_EXIT_CODE) -> None:
    """Drop-in for ``hfai.client.go_suspend()``: flush and exit for re-queue."""
    sys.stdout.flush()
    sys.stderr.flush()
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        try:
            dist.destroy_process_group()
        except Exception:
            pass
    raise SystemExit(code)
