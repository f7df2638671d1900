"""``hfai.multiprocessing.spawn(fn, args=(), nprocs=N, bind_numa=True)`` equivalent
(reference ``restnet_ddp.py:153-155``): ``fn(local_rank, *args)`` in ``nprocs`` processes, each pinned
to the CPUs of its GPU's NUMA node."""
from ..launch import spawn

__all__ = ["spawn"]
