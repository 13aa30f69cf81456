"""Checkpointable counter-based (Philox4x32-10) RNG stream for the native dropout kernels.

Every dropout launch consumes a contiguous counter range [offset, offset + ceil(n/4)) of the
stream (seed).  The state is two integers, saved in checkpoints and restored on resume so the
masks after a restart are bit-identical (BASELINE config 5); the backward pass regenerates a
mask from the (seed, offset) recorded by its forward instead of storing it.
"""
from __future__ import annotations

import threading


class PhiloxStream:
    def __init__(self, seed: int = 0x5EED, offset: int = 0):
        self.seed = int(seed) & ((1 << 64) - 1)
        self.offset = int(offset)
        self._lock = threading.Lock()

    def reserve(self, numel: int) -> tuple[int, int]:
        """Reserve counters for `numel` elements; returns (seed, offset)."""
        n = (int(numel) + 3) // 4
        with self._lock:
            off = self.offset
            self.offset += n
        return self.seed, off

    def state_dict(self) -> dict:
        return {"seed": self.seed, "offset": self.offset}

    def load_state_dict(self, sd: dict) -> None:
        self.seed = int(sd["seed"])
        self.offset = int(sd["offset"])


_default = PhiloxStream()


def default_stream() -> PhiloxStream:
    return _default


def manual_seed(seed: int) -> None:
    _default.seed = int(seed) & ((1 << 64) - 1)
    _default.offset = 0
