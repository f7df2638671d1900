"""Process launch + rendezvous: replacement for ``hfai.multiprocessing.spawn`` and
the reference's env contract.

Reference contract (``restnet_ddp.py:86-95,153-155``): the script is started
once per *node* with ``MASTER_IP``, ``MASTER_PORT``, ``WORLD_SIZE`` (= number of
nodes) and ``RANK`` (= node index); it spawns one process per visible GPU
(NUMA-bound), and each computes ``world = nodes * gpus`` and
``rank = node * gpus + local_rank``.

:func:`spawn` keeps that contract (single-node defaults: 127.0.0.1, a free
port, 1 node, node 0) and additionally pins each child to the CPUs of the NUMA
node nearest its GPU (read from sysfs). :func:`dist_env` also accepts a
``torchrun``-style launch (``LOCAL_RANK``/``LOCAL_WORLD_SIZE`` present), which is
how ``bench.py`` is driven.
"""
from __future__ import annotations

import os
import socket
from dataclasses import dataclass
from typing import Callable, Optional, Sequence

import torch

__all__ = ["DistEnv", "dist_env", "spawn", "free_port", "bind_numa", "init_distributed", "gpu_pci_bdf",
           "host_group", "visible_gpu_count"]

# KFD topology (sysfs): the GPU list in HSA agent order, readable without initialising HIP
_KFD_ROOT = "/sys/class/kfd/kfd/topology/nodes"
_DRI_ROOT = "/dev/dri"
_UNPARSED = object()   # a *_VISIBLE_DEVICES selector that is not a list of indices (UUIDs)


def _kfd_gpus():
    """Property dicts of the GPU nodes of the KFD topology (simd_count > 0) that this process may
    open, in HSA agent order; None when the topology is not readable. sysfs is not namespaced: a
    container given only some render nodes still lists every GPU of the host, so a node counts only
    when its ``/dev/dri/renderD<drm_render_minor>`` is accessible (when /dev/dri exists at all)."""
    try:
        gpus = []
        dri = os.path.isdir(_DRI_ROOT)
        for n in sorted((d for d in os.listdir(_KFD_ROOT) if d.isdigit()), key=int):
            with open(f"{_KFD_ROOT}/{n}/properties") as f:
                kv = dict(l.split(" ", 1) for l in f.read().split("\n") if " " in l)
            if int(kv.get("simd_count", "0")) <= 0:
                continue
            minor = kv.get("drm_render_minor")
            if dri and minor is not None and int(minor) > 0 and not os.access(
                    f"{_DRI_ROOT}/renderD{int(minor)}", os.R_OK | os.W_OK):
                continue
            gpus.append(kv)
        return gpus
    except (OSError, ValueError):
        return None


def _visible_list():
    """Indices (into the KFD GPU list) of the GPUs the *_VISIBLE_DEVICES variables select, or None
    when none is set. ROCR_VISIBLE_DEVICES applies first (ROCr); HIP then applies
    HIP_VISIBLE_DEVICES, or CUDA_VISIBLE_DEVICES only when HIP_VISIBLE_DEVICES is unset (HIP reads
    one of the two, not both). ``_UNPARSED`` when a selector is not a list of integers (UUIDs)."""
    sel = None
    hip = "HIP_VISIBLE_DEVICES" if "HIP_VISIBLE_DEVICES" in os.environ else "CUDA_VISIBLE_DEVICES"
    for var in ("ROCR_VISIBLE_DEVICES", hip):
        v = os.environ.get(var)
        if v is None:
            continue
        try:
            ids = [int(x) for x in v.split(",") if x.strip() != ""]
        except ValueError:
            return _UNPARSED
        sel = ids if sel is None else [sel[i] for i in ids if 0 <= i < len(sel)]
    return sel


def _child_device_count() -> int:
    """torch's device count, taken in a short-lived child process so that THIS process starts no
    HIP runtime (and its threads) before the launcher binds its NUMA node."""
    import subprocess
    import sys
    try:
        r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                           capture_output=True, text=True, timeout=300)
        return int(r.stdout.strip().splitlines()[-1])
    except (OSError, ValueError, IndexError, subprocess.SubprocessError):
        return 0


def visible_gpu_count() -> int:
    """GPUs this process will see, counted from the KFD topology and the *_VISIBLE_DEVICES
    variables -- no HIP call, so the launcher can bind a rank's NUMA node BEFORE the HIP runtime
    starts its threads (they inherit the affinity the process has then). Where the topology is
    not readable (no ROCm driver) or a selector names devices by UUID, the count comes from torch
    in a child process instead of a guess."""
    gpus = _kfd_gpus()
    sel = _visible_list() if gpus is not None else None
    if gpus is None or sel is _UNPARSED:
        return _child_device_count()
    if sel is None:
        return len(gpus)
    return sum(1 for i in sel if 0 <= i < len(gpus))


@dataclass
class DistEnv:
    master_addr: str
    master_port: int
    world_size: int
    rank: int
    local_rank: int
    local_world_size: int
    node_rank: int
    nnodes: int


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def dist_env(local_rank: Optional[int] = None, nprocs: Optional[int] = None) -> DistEnv:
    env = os.environ
    if "LOCAL_RANK" in env and local_rank is None:          # torchrun
        lr = int(env["LOCAL_RANK"])
        lws = int(env.get("LOCAL_WORLD_SIZE", env.get("WORLD_SIZE", "1")))
        world = int(env.get("WORLD_SIZE", "1"))
        rank = int(env.get("RANK", str(lr)))
        return DistEnv(env.get("MASTER_ADDR", "127.0.0.1"), int(env.get("MASTER_PORT", "29500")),
                       world, rank, lr, lws, rank // max(lws, 1), max(world // max(lws, 1), 1))
    # reference contract: WORLD_SIZE = nodes, RANK = node index
    addr = env.get("MASTER_IP", env.get("MASTER_ADDR", "127.0.0.1"))
    port = int(env.get("MASTER_PORT", "29500"))
    nnodes = int(env.get("WORLD_SIZE", "1"))
    node = int(env.get("RANK", "0"))
    lr = 0 if local_rank is None else local_rank
    gpus = nprocs if nprocs is not None else max(visible_gpu_count(), 1)
    return DistEnv(addr, port, nnodes * gpus, node * gpus + lr, lr, gpus, node, nnodes)


def gpu_pci_bdf(index: int) -> Optional[str]:
    """PCI address (``dddd:bb:dd.f``) of the ``index``-th VISIBLE GPU (KFD topology in HSA agent
    order, remapped through *_VISIBLE_DEVICES)."""
    gpus = _kfd_gpus()
    if not gpus:
        return None
    sel = _visible_list()
    if sel is _UNPARSED:
        return None
    if sel is not None:
        if not 0 <= index < len(sel):
            return None
        index = sel[index]
    if not 0 <= index < len(gpus):
        return None
    try:
        dom = int(gpus[index].get("domain", "0"))
        loc = int(gpus[index].get("location_id", "0"))
    except ValueError:
        return None
    return f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7}"


def _gpu_numa_cpus(local_rank: int) -> Optional[Sequence[int]]:
    """CPUs of the NUMA node that hosts GPU ``local_rank`` (KFD topology, sysfs)."""
    try:
        bdf = gpu_pci_bdf(local_rank)
        if bdf is None:
            return None
        numa = int(open(f"/sys/bus/pci/devices/{bdf}/numa_node").read())
        if numa < 0:
            return None
        cpulist = open(f"/sys/devices/system/node/node{numa}/cpulist").read().strip()
        cpus = []
        for part in cpulist.split(","):
            a, _, b = part.partition("-")
            cpus.extend(range(int(a), int(b or a) + 1))
        return cpus
    except (OSError, ValueError, KeyError):
        return None


def bind_numa(local_rank: int) -> bool:
    """Pin this process to the CPUs of GPU ``local_rank``'s NUMA node (intersected with the CPUs
    it may already use, so a cgroup cpuset is respected); False when nothing was changed."""
    cpus = _gpu_numa_cpus(local_rank)
    if not cpus:
        return False
    try:
        allowed = os.sched_getaffinity(0)
        cpus = sorted(set(cpus) & allowed)
        if not cpus or set(cpus) == allowed:
            return False
        os.sched_setaffinity(0, cpus)
        return True
    except OSError:
        return False


def _child(local_rank: int, fn: Callable, args: tuple, numa: bool) -> None:
    if numa:
        bind_numa(local_rank)
    fn(local_rank, *args)


def spawn(fn: Callable, args: tuple = (), nprocs: Optional[int] = None, bind_numa: bool = True,
          join: bool = True):
    """``hfai.multiprocessing.spawn`` equivalent: ``fn(local_rank, *args)`` in ``nprocs`` procs."""
    import torch.multiprocessing as mp
    nprocs = nprocs if nprocs is not None else max(visible_gpu_count(), 1)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if "MASTER_PORT" not in os.environ:
        os.environ["MASTER_PORT"] = str(free_port())
    os.environ.setdefault("MASTER_IP", os.environ.get("MASTER_ADDR", "127.0.0.1"))
    bind_numa = bind_numa and os.environ.get("PDA_BIND_NUMA", "1") != "0"
    if nprocs == 1:
        _child(0, fn, args, bind_numa)
        return None
    return mp.spawn(_child, args=(fn, args, bind_numa), nprocs=nprocs, join=join)


_HOST_GROUP = None


def host_group():
    """Process group for HOST-side collectives (suspend flag, validation counters, barriers, bench
    bookkeeping): gloo over TCP. Device collectives go through the framework's own RCCL
    communicator (:mod:`~pytorch_distributed_amd.parallel.rccl`), so each process holds ONE RCCL
    communicator: torch's NCCL process group is only the rendezvous (its communicator is created
    lazily, i.e. never). Must be called by every rank (it creates the group collectively the first
    time); :func:`init_distributed` does so."""
    global _HOST_GROUP
    import torch.distributed as dist
    if _HOST_GROUP is None:
        _HOST_GROUP = (dist.group.WORLD if dist.get_backend() == "gloo"
                       else dist.new_group(backend="gloo"))
    return _HOST_GROUP


def init_distributed(env: DistEnv, backend: str, timeout_s: float = 1800.0,
                     device: Optional[torch.device] = None) -> None:
    """TCP rendezvous (reference ``restnet_ddp.py:94``) + the gloo host group. The gradient
    communicator is the framework's native RCCL one (created by DistributedDataParallel), so no
    ``device_id`` here: torch's own NCCL communicator is never instantiated."""
    import datetime
    import torch.distributed as dist
    if dist.is_initialized():
        return
    dist.init_process_group(backend=backend,
                            init_method=f"tcp://{env.master_addr}:{env.master_port}",
                            world_size=env.world_size, rank=env.rank,
                            timeout=datetime.timedelta(seconds=timeout_s))
    host_group()
