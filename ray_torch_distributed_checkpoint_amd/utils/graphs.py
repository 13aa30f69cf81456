"""Whole-step hipGraph capture for launch-bound training steps.

The reference toy model (R/my_ray_module.py:94-112, B = 16 per worker) is far below MFMA
saturation: its step is ~15 kernel launches of a few microseconds each, so the step time is
launch latency.  `CapturedStep` records one complete step - zero_grad,
forward, loss, backward, optimizer - into a hipGraph (torch.cuda.CUDAGraph is hipGraph on
ROCm) and replays it with a single launch.  Every native op runs on the current stream and
allocates from torch's caching allocator, so capture works unchanged; the pieces of host
state a replay would otherwise freeze are made device-resident:

* dropout: the Philox counter base moves to a device int64 (ops/random.PhiloxStream graph
  mode) and the captured step ends with `base += consumed`, so each replay draws new masks
  that are bit-identical to the eager sequence;
* gradients: the flat buffer is overwritten in place every step (ops/gradbuf), no memset;
* optimizer: FusedSGD (constant lr) is graph-safe; FusedAdamW's bias correction is a host
  scalar per step, so it refuses capture.

Inputs must be static tensors: copy each new batch into `step.inputs[...]` before `replay()`.

    step = CapturedStep(lambda: train_step(static_x, static_y), warmup=3)
    for x, y in loader:
        static_x.copy_(x); static_y.copy_(y)
        loss = step.replay()
"""
from __future__ import annotations

import torch

from ..ops.random import PhiloxStream, default_stream


class CapturedStep:
    def __init__(self, fn, warmup: int = 3, philox: PhiloxStream | None = None, pool=None):
        if not torch.cuda.is_available():
            raise RuntimeError("hipGraph capture needs a GPU")
        self.fn = fn
        self.philox = philox or default_stream()
        dev = torch.cuda.current_device()
        from ..ops.streams import side_stream

        side = side_stream(dev, "capture")
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # warm-up: lazy allocations, optimizer state, workspaces
            for _ in range(warmup):
                fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        # several captured steps (e.g. one per input batch) share the device counter base: the
        # first capture enters graph mode, the others reuse it (each ends with base += consumed);
        # graph mode is reference-counted and ends when the last of them is closed
        self.philox.acquire_graph_mode(dev)
        self._holds_philox = True
        self.graph = torch.cuda.CUDAGraph()
        try:
            # capture on the reserved stream, not torch.cuda.graph's own pool stream (which
            # may alias another user's handle, e.g. the checkpoint engine's copy stream)
            with torch.cuda.graph(self.graph, pool=pool, stream=side):
                self.out = fn()
                self.philox.end_graph_step()
        except Exception:
            self._holds_philox = False
            self.philox.release_graph_mode()
            raise
        self.replays = 0

    def replay(self):
        self.graph.replay()
        self.replays += 1
        return self.out

    def close(self) -> None:
        """Release this capture's share of Philox graph mode; when the last live capture closes,
        the host counter resumes where the replays left it (an owner closing first no
        longer frees the device base other captures still replay against)."""
        torch.cuda.synchronize()
        if getattr(self, "_holds_philox", False):
            self._holds_philox = False
            self.philox.release_graph_mode()
