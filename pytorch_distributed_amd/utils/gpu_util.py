"""Average GPU utilisation over a timed region -- the reference's "Avg GPU Util" panel
(``/root/reference/README.md:33-40``, ``result.png``), which its authors read from cluster
monitoring (nvidia-smi style: the fraction of time a kernel was executing).

The amdgpu driver exposes the same quantity as ``gpu_busy_percent`` in the GPU's PCI sysfs
directory (what ``rocm-smi --showuse`` prints). :class:`BusySampler` polls it on a daemon thread
every ``interval`` seconds while a region runs and reports the mean per device (None where the file
is not readable, e.g. a container without the device's sysfs)."""
from __future__ import annotations

import threading
import time
from typing import Dict, List, Optional, Sequence

from ..launch import gpu_pci_bdf

__all__ = ["BusySampler", "StepBusy", "busy_path", "kernel_busy"]


def busy_path(index: int) -> Optional[str]:
    bdf = gpu_pci_bdf(index)
    if bdf is None:
        return None
    path = f"/sys/bus/pci/devices/{bdf}/gpu_busy_percent"
    try:
        int(open(path).read().strip())
    except (OSError, ValueError):
        return None
    return path


class BusySampler:
    def __init__(self, devices: Sequence[int], interval: float = 0.01) -> None:
        self.devices = list(devices)
        self.paths = [busy_path(d) for d in self.devices]
        self.interval = interval
        self.samples: List[List[int]] = [[] for _ in self.devices]
        self._stop = threading.Event()
        self._thr: Optional[threading.Thread] = None

    def _run(self) -> None:
        while not self._stop.is_set():
            for i, p in enumerate(self.paths):
                if p is None:
                    continue
                try:
                    self.samples[i].append(int(open(p).read().strip()))
                except (OSError, ValueError):
                    pass
            time.sleep(self.interval)

    def __enter__(self) -> "BusySampler":
        if any(self.paths):
            self._thr = threading.Thread(target=self._run, daemon=True)
            self._thr.start()
        return self

    def __exit__(self, *exc) -> None:
        self._stop.set()
        if self._thr is not None:
            self._thr.join()

    def mean(self) -> Dict[int, Optional[float]]:
        return {d: (round(sum(s) / len(s), 1) if s else None) for d, s in zip(self.devices, self.samples)}

    def overall(self) -> Optional[float]:
        v = [x for x in self.mean().values() if x is not None]
        return round(sum(v) / len(v), 1) if v else None


class StepBusy:
    """Device-busy % where the sysfs counter is not readable: HIP events on the compute stream at
    the start and end of every training step (``begin`` / ``end``), read after the step's
    synchronize, summed over the region and divided by its wall time. The trainer synchronises
    after every step (as the reference), so the intervals do not overlap and the remainder is the
    time the device waits for the host; within a step the kernels keep the device busy (98.6 % by
    the kernel-interval union, ``bench.py``), so this slightly over-counts, never under."""

    def __init__(self, device) -> None:
        import torch
        self.on = device is not None and device.type == "cuda"
        self.device = device
        self._t = torch
        self.dev_ms = 0.0
        self.wall_s = 0.0
        self._pending = []
        self._e0 = None

    def __enter__(self) -> "StepBusy":
        self._w0 = time.perf_counter()
        return self

    def __exit__(self, *exc) -> None:
        if self.on:
            self._t.cuda.synchronize(self.device)
            self._collect()
        self.wall_s += time.perf_counter() - self._w0

    def begin(self) -> None:
        if self.on:
            self._e0 = self._t.cuda.Event(enable_timing=True)
            self._e0.record(self._t.cuda.current_stream(self.device))

    def end(self) -> None:
        if self.on and self._e0 is not None:
            e1 = self._t.cuda.Event(enable_timing=True)
            e1.record(self._t.cuda.current_stream(self.device))
            self._pending.append((self._e0, e1))
            self._e0 = None
            if len(self._pending) > 64:
                self._collect()

    def _collect(self) -> None:
        keep = []
        for a, b in self._pending:
            if b.query():
                self.dev_ms += a.elapsed_time(b)
            else:
                keep.append((a, b))
        self._pending = keep

    def overall(self) -> Optional[float]:
        if not self.on or self.wall_s <= 0 or self.dev_ms <= 0:
            return None
        return round(min(100.0, 100.0 * self.dev_ms / (1e3 * self.wall_s)), 1)


def kernel_busy(step_fn, steps: int, devices: Sequence[int]) -> Dict[int, Optional[float]]:
    """Device-busy % measured from the kernels themselves, for hosts where the driver's sysfs
    counter is not readable (e.g. inside a container): ``steps`` calls of ``step_fn(i)`` under
    torch.profiler (ROCm: roctracer kernel records), then per device the union of kernel intervals
    over the span from its first kernel start to its last kernel end -- the same quantity
    (fraction of time any kernel is running) that ``gpu_busy_percent`` samples."""
    import torch
    from torch.autograd import DeviceType
    from torch.profiler import ProfilerActivity, profile
    for d in devices:
        torch.cuda.synchronize(d)
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        for i in range(steps):
            step_fn(i)
        for d in devices:
            torch.cuda.synchronize(d)
    # ROCTracer labels device records with the HSA agent index (CPU agents first), not the torch
    # device index: agents are mapped onto the requested devices in enumeration order
    by_agent: Dict[int, list] = {}
    for e in prof.events():
        if e.device_type != DeviceType.CUDA or e.time_range.end <= e.time_range.start:
            continue
        by_agent.setdefault(e.device_index, []).append((e.time_range.start, e.time_range.end))
    per: Dict[int, list] = {d: [] for d in devices}
    agents = sorted(by_agent)
    if len(devices) == 1:
        per[devices[0]] = [iv for a in agents for iv in by_agent[a]]
    elif len(agents) == len(devices):
        for d, a in zip(sorted(devices), agents):
            per[d] = by_agent[a]
    out: Dict[int, Optional[float]] = {}
    for d, iv in per.items():
        if not iv:
            out[d] = None
            continue
        iv.sort()
        busy, cs, ce = 0, iv[0][0], iv[0][1]
        for s_, e_ in iv[1:]:
            if s_ > ce:
                busy += ce - cs
                cs, ce = s_, e_
            else:
                ce = max(ce, e_)
        busy += ce - cs
        span = iv[-1][1] - iv[0][0]
        out[d] = round(100.0 * busy / span, 1) if span > 0 else None
    return out
