"""Checkpointable counter-based (Philox4x32-10) RNG stream for the native dropout kernels.

Every dropout launch consumes a contiguous counter range [offset, offset + ceil(n/4)) of the
stream (seed).  The state is two integers, saved in checkpoints and restored on resume so the
masks after a restart are bit-identical (BASELINE config 5); the backward pass regenerates a
mask from the (seed, offset) recorded by its forward instead of storing it.
"""
from __future__ import annotations

import threading


class PhiloxStream:
    """In graph mode (a captured hipGraph step, utils/graphs.py) the counter base lives in a
    device int64 (`device_base`): kernels add it to the step-relative offsets recorded at
    capture time, and the captured step ends with `base += consumed`, so every replay draws
    fresh masks while the host never runs."""

    def __init__(self, seed: int = 0x5EED, offset: int = 0):
        self.seed = int(seed) & ((1 << 64) - 1)
        self.offset = int(offset)
        self._lock = threading.Lock()
        self._base = None  # device counter base in graph mode
        self._graph_users = 0  # live captured steps sharing _base (acquire/release_graph_mode)

    def device_base(self):
        return self._base

    def enter_graph_mode(self, device) -> None:
        import torch

        self._base = torch.tensor([self.offset], dtype=torch.int64, device=device)
        self.offset = 0

    def end_graph_step(self) -> None:
        """Called inside the capture after the step's last dropout: advance the device base."""
        self._base.add_(self.offset)
        self.offset = 0

    def exit_graph_mode(self) -> None:
        if self._base is not None:
            self.offset = int(self._base.item()) + self.offset
            self._base = None
        self._graph_users = 0

    def acquire_graph_mode(self, device) -> None:
        """A captured step starts using the device base: the first user enters graph mode, the
        others share it (each of their graphs ends with base += consumed)."""
        if self._base is None:
            self.enter_graph_mode(device)
            self._graph_users = 0
        self._graph_users += 1

    def release_graph_mode(self) -> None:
        """A captured step is closed: graph mode ends with the LAST user, so no live graph ever
        replays against a freed device base (or a host offset that overlaps its counter)."""
        if self._graph_users > 0:
            self._graph_users -= 1
            if self._graph_users == 0:
                self.exit_graph_mode()

    def reserve(self, numel: int) -> tuple[int, int]:
        """Reserve counters for `numel` elements; returns (seed, offset)."""
        n = (int(numel) + 3) // 4
        with self._lock:
            off = self.offset
            self.offset += n
        return self.seed, off

    def state_dict(self) -> dict:
        off = self.offset if self._base is None else int(self._base.item()) + self.offset
        return {"seed": self.seed, "offset": off}

    def load_state_dict(self, sd: dict) -> None:
        self.seed = int(sd["seed"])
        if self._base is not None:
            self._base.fill_(int(sd["offset"]))
            self.offset = 0
        else:
            self.offset = int(sd["offset"])


_default = PhiloxStream()


def default_stream() -> PhiloxStream:
    return _default


def manual_seed(seed: int) -> None:
    _default.seed = int(seed) & ((1 << 64) - 1)
    _default.offset = 0
