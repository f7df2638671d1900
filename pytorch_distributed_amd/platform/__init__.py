"""The reference's platform API (High-Flyer ``hfai``), re-homed on this framework.

The reference scripts reach their dataset, preemption client, launcher, DDP wrapper and NCCL
wrapper through ``hfai`` (e.g. ``restnet_ddp.py:12-16, 101-119, 35-47,
153-155``). This package exposes the same names with the same call signatures, backed by this
repository's components, so a script written against the reference ports by changing imports::

    import pytorch_distributed_amd.platform as hfai
    import pytorch_distributed_amd.platform.nccl.distributed as dist
    from pytorch_distributed_amd.platform.nn.parallel import DistributedDataParallel

| hfai name                                     | here                                            |
|-----------------------------------------------|-------------------------------------------------|
| ``hfai.datasets.ImageNet(split, transform)``  | :func:`datasets.ImageNet` (synthetic / folder)  |
| ``hfai.client.receive_suspend_command()``     | :mod:`client` (signal / sentinel / step trigger)|
| ``hfai.client.go_suspend()``                  | :mod:`client` (exit with the requeue code)      |
| ``hfai.multiprocessing.spawn(..., bind_numa)``| :mod:`multiprocessing` (NUMA-pinned children)   |
| ``hfai.nn.parallel.DistributedDataParallel``  | :mod:`nn.parallel` (RCCL bucket reducer)        |
| ``hfai.nccl.distributed``                     | :mod:`nccl.distributed` (torch.distributed, RCCL)|
"""
from . import client, datasets, multiprocessing, nccl, nn  # noqa: F401

__all__ = ["client", "datasets", "multiprocessing", "nccl", "nn"]
