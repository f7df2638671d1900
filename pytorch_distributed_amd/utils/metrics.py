"""Throughput / timing helpers and the opt-in JSONL metrics log."""
from __future__ import annotations

import json
import time
from pathlib import Path
from typing import Optional

import torch

__all__ = ["Throughput", "MetricsLog", "gpu_mem_gb"]


def gpu_mem_gb() -> float:
    if torch.cuda.is_available():
        return torch.cuda.max_memory_allocated() / 1e9
    return 0.0


class Throughput:
    """Images/sec with warm-up exclusion, timed on the host between device syncs."""

    def __init__(self, warmup: int = 0) -> None:
        self.warmup = warmup
        self.steps = 0
        self.images = 0
        self.t0: Optional[float] = None
        self.elapsed = 0.0

    def _sync(self) -> None:
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    def step(self, batch: int) -> None:
        self.steps += 1
        if self.steps == self.warmup:
            self._sync()
            self.t0 = time.perf_counter()
        elif self.steps > self.warmup:
            if self.t0 is None:
                self.t0 = time.perf_counter()
            self.images += batch

    def rate(self) -> float:
        if self.t0 is None or self.images == 0:
            return 0.0
        self._sync()
        self.elapsed = time.perf_counter() - self.t0
        return self.images / self.elapsed


class StepProfiler:
    """``MX_PROFILE=<n>``: record the first n training steps with torch.profiler (ROCm kernel
    names are our HIP kernels) and write a chrome trace to ``<save_path>/profile_rank<r>.json``.
    For hardware counters use ``tools/gpu_profile.sh`` (rocprofv3) instead."""

    def __init__(self, steps: int, out_dir, rank: int = 0) -> None:
        self.steps = steps
        self.n = 0
        self.out = Path(out_dir) / f"profile_rank{rank}.json"
        self.prof = None
        if steps > 0:
            acts = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self.prof = torch.profiler.profile(activities=acts)
            self.prof.__enter__()

    def step(self) -> None:
        if self.prof is None:
            return
        self.n += 1
        if self.n >= self.steps:
            self.close()

    def close(self) -> None:
        if self.prof is None:
            return
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self.prof.__exit__(None, None, None)
        self.out.parent.mkdir(parents=True, exist_ok=True)
        self.prof.export_chrome_trace(str(self.out))
        self.prof = None


class MetricsLog:
    def __init__(self, path, enabled: bool = True) -> None:
        self.path = Path(path)
        self.enabled = enabled
        if enabled:
            self.path.parent.mkdir(parents=True, exist_ok=True)

    def write(self, **kw) -> None:
        if not self.enabled:
            return
        kw.setdefault("ts", time.time())
        with open(self.path, "a") as f:
            f.write(json.dumps(kw) + "\n")
