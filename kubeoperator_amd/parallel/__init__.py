"""Parallelism for the bundled training chart: flat bucketed parameter storage, RCCL data parallelism
(DDP all-reduce or ZeRO-1 reduce-scatter/all-gather), process-group bootstrap."""
from .ddp import DataParallel
from .dist import DistInfo, barrier, init_distributed, shutdown
from .flat import Bucket, FlatParamStore, ParamSpec

__all__ = ["DataParallel", "DistInfo", "barrier", "init_distributed", "shutdown", "Bucket", "FlatParamStore",
           "ParamSpec"]
