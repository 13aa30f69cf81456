"""Communicator health: a timed-out collective must never reach an optimizer step or a checkpoint.

The one-shot P2P all-reduce (parallel/p2p.py) waits for its peers with a bounded spin.  On a
timeout it fills the bucket with NaN and sets a host-coherent error word, because leaving the
local, un-reduced gradient in place would let ranks silently diverge.  That word is the single
source of truth for "this rank's gradients are poisoned", and three places consult it:

* **the device**: the fused AdamW / SGD kernels take its address (`skip_ptr`) and turn the
  update into a no-op when it is set (kernels/optim.hip `comm_poisoned`).  This is the only
  guard that also holds inside a replayed hipGraph, where no host code runs between the
  collective and the step;
* **the host, per step**: `DistributedDataParallel._finalize` and the captured-step replay in
  my_ray_module raise as soon as the word is visible;
* **every checkpoint write**: `assert_healthy()` synchronises the device and raises before any
  snapshot is taken (checkpoint/dcp.py save/async_save, checkpoint/torchsave.py save), so a
  poisoned state is never staged, let alone committed.  A supervisor restart then resumes from
  the last committed (clean) checkpoint (train/launcher.py).

The reference has none of this (R/my_ray_module.py:155-160 relies on NCCL's own watchdog).
"""
from __future__ import annotations

import weakref

import torch


class CommPoisonedError(RuntimeError):
    """A gradient collective timed out waiting for a peer; this rank's gradients are NaN."""


_comms: "weakref.WeakSet" = weakref.WeakSet()


def register(comm) -> None:
    """Track a communicator that exposes `error() -> int` and `error_ptr() -> int`."""
    _comms.add(comm)


def unregister(comm) -> None:
    _comms.discard(comm)


def active() -> bool:
    return len(_comms) > 0


def error() -> int:
    """Non-zero when any registered communicator recorded a timeout (reads host-coherent words;
    a collective still running on the device may set one later)."""
    return next((e for e in (c.error() for c in list(_comms)) if e), 0)


def assert_healthy(what: str = "checkpoint", sync: bool = True) -> None:
    """Raise CommPoisonedError if a gradient collective of this process timed out.  With `sync`
    the device is synchronised first, so every collective enqueued before this call has either
    completed or recorded its timeout."""
    if not _comms:
        return
    if sync and torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()
    if error():
        raise CommPoisonedError(f"refusing {what}: a P2P gradient all-reduce timed out waiting for a peer rank "
                                "(gradients were poisoned with NaN and the optimizer skipped its update)")
