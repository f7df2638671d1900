from .comm import Communicator, ProcessGroupCommunicator, make_communicator
from .ddp import DistributedDataParallel, NativeReducer
from .dp import DataParallel
from .reducer import Reducer, plan_buckets

__all__ = ["Communicator", "ProcessGroupCommunicator", "make_communicator",
           "DistributedDataParallel", "NativeReducer", "DataParallel", "Reducer", "plan_buckets"]
