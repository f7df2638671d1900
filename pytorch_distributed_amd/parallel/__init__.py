from .comm import Communicator, ProcessGroupCommunicator, make_communicator
from .ddp import DistributedDataParallel, NativeReducer, convert_sync_batchnorm
from .dp import DataParallel
from .reducer import Reducer, plan_buckets

__all__ = ["Communicator", "ProcessGroupCommunicator", "make_communicator",
           "DistributedDataParallel", "NativeReducer", "convert_sync_batchnorm", "DataParallel",
           "Reducer", "plan_buckets"]
