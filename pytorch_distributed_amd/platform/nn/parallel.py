"""``hfai.nn.parallel`` equivalent: ``DistributedDataParallel(module, device_ids=None)`` (reference
``restnet_ddp.py:99``, ``resnet_ddp_apex.py:103``) and ``DataParallel``."""
from ...parallel.ddp import DistributedDataParallel
from ...parallel.dp import DataParallel

__all__ = ["DistributedDataParallel", "DataParallel"]
