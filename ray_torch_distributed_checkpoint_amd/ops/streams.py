"""Process-wide side streams, one per user and device, created once.

A MI355X process gets GPU_MAX_HW_QUEUES (4) hardware queues; HIP streams beyond that share
queues round-robin, and a side stream that lands on the compute stream's queue serialises
with it.  Every side stream of the framework's compute path is made here (the DDP widen / P2P
streams in csrc/runtime/reducer.cpp `shared_stream`), once per process, so re-wrapping a model
or re-running a step never adds streams.

Users: "wgrad" (the grouped weight-gradient GEMMs, ops/gemm.py), "sort" (the embedding
backward's token sort, ops/embedding.py), "ckpt" (the checkpoint engine's copy stream,
checkpoint/torchsave.py), "overlap" (optim/overlap.py), "h2d" / "dataset_h2d" (input copies),
"capture" (hipGraph warm-up and capture, utils/graphs.py, my_ray_module.py).  The Stream objects
live here for the process lifetime, and each user key draws its own entry of PyTorch's stream
pool, so no two framework users alias one hipStream_t (the pool hands a handle out again only
after 32 requests).  RTDC_SHARED_SIDE=1 gives "wgrad" and "sort" one stream: neutral
on one GPU (17.22 vs 17.24 ms GPT-2 step) but +0.7 ms under DDP (18.35 / 18.27 vs 17.51 /
17.68 ms, 1-rank RCCL, r4; the bucket collectives are launched from the wgrad stream's
gradient-ready callbacks - which ordering costs the time was not isolated).
"""
from __future__ import annotations

import os

import torch

_side: dict = {}
_SHARED = os.environ.get("RTDC_SHARED_SIDE", "0") == "1"  # 1: one stream for all users (A/B)


def side_stream(device, user: str = "") -> torch.cuda.Stream:
    """The device's compute side stream (created once)."""
    device = torch.device(device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    key = (idx, "" if _SHARED and user in ("wgrad", "sort") else user)
    s = _side.get(key)
    if s is None:
        s = torch.cuda.Stream(device=torch.device("cuda", idx))
        _side[key] = s
    return s
