"""Data parallelism: the DDP wrapper over the native gradient-bucket engine (RCCL all-reduce
overlapped with backward) and the seed+epoch sharded sampler."""
from .ddp import DistributedDataParallel
from .sampler import DistributedSampler

__all__ = ["DistributedDataParallel", "DistributedSampler"]
