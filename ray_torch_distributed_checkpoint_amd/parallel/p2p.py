"""One-shot intra-node all-reduce over hipIpc-mapped peer buffers.

RCCL's ring all-reduce is latency-bound for small buckets: 2(N-1) dependent hops on
point-to-point xGMI.  Here every rank copies its bucket into an exported, uncached staging
buffer, publishes an epoch flag, and each rank then reads all N staging buffers at once (all 7
links of an MI355X in parallel, one hop) and sums them in rank order - bitwise the same result on
every rank, deterministic run to run.  Native kernel + protocol: csrc/kernels/p2p_allreduce.hip,
communicator: csrc/runtime/p2p_comm.cpp.  The gradient-bucket engine routes buckets at or below
`max_bytes` here (parallel/ddp.py `p2p_max_kb`); larger ones stay on RCCL.

Requirements: every rank of the group on one node with its own GPU (or, for tests, several
processes sharing one GPU), the dmabuf IPC mode (HSA_ENABLE_IPC_MODE_LEGACY=0), ≤ 8 ranks.
Waits are bounded (`timeout_s`): a missing peer raises on the next call instead of hanging.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops._ext import gpu_ext


class P2PAllReduce:
    def __init__(self, group=None, capacity_mb: float = 4.0, device=None, timeout_s: float = 30.0,
                 blocks: int = 32):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if self.world > 8:
            raise ValueError("P2PAllReduce: at most 8 ranks (one node)")
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        cap = int(capacity_mb * (1 << 20))
        self.comm = gpu_ext().P2PComm(self.rank, self.world, cap, dev.index, float(timeout_s), int(blocks))
        handles = [None] * self.world
        dist.all_gather_object(handles, bytes(self.comm.handle()), group=group)
        self.comm.open(handles)
        self.device = dev
        from . import health

        health.register(self)  # checkpoints refuse to snapshot after a timeout (parallel/health.py)

    @property
    def capacity(self) -> int:
        return self.comm.capacity()

    def all_reduce_(self, t: torch.Tensor, average: bool = True) -> torch.Tensor:
        """In-place all-reduce (sum, or mean when average) of a contiguous fp32/bf16 tensor of at
        most `capacity` bytes on the current stream."""
        self.comm.allreduce_(t, average)
        return t

    def error(self) -> int:
        return self.comm.error()

    def error_ptr(self) -> int:
        """Device-readable address of the error word (the fused optimizers' `skip_ptr`)."""
        return self.comm.error_ptr()

    def snapshot_error(self, dst: torch.Tensor, idx: int) -> None:
        """Copy the error word into dst[idx] (pinned int32), ordered on the current stream."""
        self.comm.snapshot_error(dst, int(idx))
