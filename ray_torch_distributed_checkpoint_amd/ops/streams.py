"""Process-wide side streams.

A MI355X process gets GPU_MAX_HW_QUEUES (4) hardware queues; HIP streams beyond that share
queues round-robin, and a side stream that lands on the compute stream's queue serialises
with it (its event waits park the compute kernels queued behind them).  A data-parallel
GPT-2 step already uses the compute stream, RCCL's stream and the DDP widen stream
(csrc/runtime/reducer.cpp `shared_stream`), so the framework's own side work - the grouped
weight-gradient GEMMs (ops/gemm.py) and the embedding backward's token sort
(ops/embedding.py) - shares ONE stream per device instead of one each: four queues, four
streams.  The sort runs under the cross-entropy kernel, long before the first grouped
weight-gradient flush, so in-order sharing costs nothing.
"""
from __future__ import annotations

import torch

_side: dict = {}


def side_stream(device) -> torch.cuda.Stream:
    """The device's compute side stream (created once)."""
    device = torch.device(device)
    key = device.index if device.index is not None else torch.cuda.current_device()
    s = _side.get(key)
    if s is None:
        s = torch.cuda.Stream(device=torch.device("cuda", key))
        _side[key] = s
    return s
