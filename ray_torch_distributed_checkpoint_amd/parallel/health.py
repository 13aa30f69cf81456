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
* **every checkpoint write**: a save refuses up front when the word is already set
  (`assert_healthy(sync=False)`: no device sync on the non-blocking path), and it records the
  word AT ITS SNAPSHOT (`capture_error_words()`: a stream-ordered copy of each communicator's
  word into pinned host memory, enqueued right after the snapshot copies).  Commit-or-refuse is
  decided from that captured value once the drain is done (`poisoned(words)`), not from the live
  sticky word: a timeout of a LATER step that happens while this snapshot drains does not void
  this clean checkpoint, and a timeout among the collectives the snapshot depends on always
  does.  A supervisor restart then resumes from the last committed (clean) checkpoint
  (train/launcher.py);
* **report()** without a checkpoint synchronises (`assert_healthy(sync=True)`) before the
  commit barrier, so a poisoned rank fails there even when it saves nothing.

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


class CapturedErrorWords:
    """Every registered communicator's error word as it stood at a point of the current stream
    (capture_error_words).  `value()` waits for the stream to pass that point (its own event) and
    returns the first non-zero word, else 0."""

    def __init__(self, words: torch.Tensor, event):
        self.words, self.event = words, event

    def value(self) -> int:
        if self.event is not None:
            self.event.synchronize()
        return next((int(w) for w in self.words.tolist() if w), 0)


def capture_error_words():
    """Enqueue, on the current stream, a copy of every registered communicator's error word into
    pinned host memory; returns a CapturedErrorWords (None when no communicator is registered).
    A save calls it right after its snapshot copies: the words then record the outcome of exactly
    the collectives the snapshot depends on."""
    comms = list(_comms)
    if not comms:
        return None
    on_dev = torch.cuda.is_available() and torch.cuda.is_initialized()
    words = torch.zeros(len(comms), dtype=torch.int32, pin_memory=on_dev)
    event = None
    for i, c in enumerate(comms):
        snap = getattr(c, "snapshot_error", None)
        if snap is not None and on_dev:
            snap(words, i)
        else:  # no stream-ordered copy available: the host-visible value now
            words[i] = int(c.error())
    if on_dev:
        event = torch.cuda.Event()
        event.record()
    return CapturedErrorWords(words, event)


def poisoned(captured) -> int:
    """Non-zero when a CapturedErrorWords recorded a timeout (None: nothing was registered)."""
    return 0 if captured is None else captured.value()


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
