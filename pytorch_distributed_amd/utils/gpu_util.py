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

__all__ = ["BusySampler", "busy_path"]


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
