"""A small columnar batch-inference dataset (the Ray Data surface used by the eval flow):
`from_items(...)` -> `.map_batches(fn, batch_size, concurrency, num_gpus)` -> `.take_all()`,
`.to_pandas()`, `.count()` (R/eval_flow.py:83-91, R/my_ray_module.py:48-50,69-72).

Blocks are numpy columns (no per-row Python objects), batches are zero-copy column slices.
Output row order equals input order, so the reference's positional `pd.concat` join
(R/eval_flow.py:91) is well defined here.

`map_batches` with a device predictor (an object with `.device` on the GPU, an
`.input_column` and `.predict_tensors(x) -> {name: device tensor}`, e.g.
my_ray_module.TorchPredictor) runs a pinned, double-buffered pipeline instead of calling the
numpy `__call__` per batch: batch i+1 is copied into one of two pinned staging buffers and
sent H2D on a side stream while batch i computes on the compute stream, outputs stay on the
device, and there is ONE device->host copy per output column at the end (the reference does a
blocking H2D + D2H per 512-row batch).  `concurrency=k` with a predictor CLASS and k visible
GPUs builds k replicas (`device=cuda:i` constructor kwarg) and shards the rows across them,
one host thread per GPU (Ray Data's actor pool, R/eval_flow.py:85-90).
"""
from __future__ import annotations

from typing import Any, Callable

import numpy as np


class Dataset:
    def __init__(self, columns: dict[str, np.ndarray]):
        n = {len(v) for v in columns.values()}
        if len(n) > 1:
            raise ValueError("columns have different lengths")
        self._cols = columns
        self._n = n.pop() if n else 0

    # ---- inspection
    def count(self) -> int:
        return self._n

    def columns(self) -> list[str]:
        return list(self._cols)

    def schema(self) -> dict:
        return {k: (v.dtype, v.shape[1:]) for k, v in self._cols.items()}

    def iter_batches(self, batch_size: int = 256):
        for s in range(0, self._n, batch_size):
            yield {k: v[s:s + batch_size] for k, v in self._cols.items()}

    def take_all(self) -> list[dict]:
        keys = list(self._cols)
        return [{k: self._cols[k][i] for k in keys} for i in range(self._n)]

    def take(self, n: int = 20) -> list[dict]:
        keys = list(self._cols)
        return [{k: self._cols[k][i] for k in keys} for i in range(min(n, self._n))]

    def to_pandas(self):
        import pandas as pd

        data = {}
        for k, v in self._cols.items():
            data[k] = list(v) if v.ndim > 1 else v
        return pd.DataFrame(data)

    def to_numpy(self) -> dict:
        return dict(self._cols)

    # ---- transforms
    def map_batches(self, fn: Callable | type, *, batch_size: int = 4096, concurrency: int | None = None,
                    num_gpus: float | None = None, fn_constructor_args: tuple = (), fn_constructor_kwargs: dict | None = None,
                    batch_format: str = "numpy", **_ignored) -> "Dataset":
        kw = dict(fn_constructor_kwargs or {})
        if isinstance(fn, type):
            k = max(1, int(concurrency or 1))
            ngpu = _gpu_count() if num_gpus else 0
            if k > 1 and ngpu >= 2 and _accepts_device(fn):
                reps = [fn(*fn_constructor_args, **dict(kw, device=f"cuda:{i}")) for i in range(min(k, ngpu))]
                return self._map_device_replicas(reps, batch_size)
            fn = fn(*fn_constructor_args, **kw)
        if _is_device_predictor(fn):
            return Dataset(self._map_device(fn, batch_size, 0, self._n))
        outs: list[dict[str, Any]] = []
        for batch in self.iter_batches(batch_size):
            outs.append(fn(batch))
        if not outs:
            return Dataset({})
        keys = list(outs[0])
        return Dataset({k: np.concatenate([np.asarray(o[k]) for o in outs]) for k in keys})

    def _map_device(self, fn, batch_size: int, lo: int, hi: int) -> dict:
        """Pinned double-buffered H2D on a side stream, compute on the current stream, outputs
        kept on the device, one D2H per output column at the end."""
        import torch

        dev = torch.device(fn.device)
        col = self._cols[getattr(fn, "input_column", "features")]
        dtype = getattr(fn, "input_dtype", torch.float32)
        B = int(batch_size)
        outs: dict[str, list] = {}
        with torch.cuda.device(dev):
            stage = [torch.empty((B,) + col.shape[1:], dtype=dtype).pin_memory() for _ in range(2)]
            views = [st.numpy() for st in stage]
            from ..ops.streams import side_stream

            h2d = side_stream(dev, "dataset_h2d")
            landed = [None, None]
            compute = torch.cuda.current_stream(dev)
            for i, s in enumerate(range(lo, hi, B)):
                k, n = i % 2, min(B, hi - s)
                if landed[k] is not None:
                    landed[k].synchronize()  # this staging buffer's previous H2D has completed
                np.copyto(views[k][:n], col[s:s + n], casting="unsafe")
                with torch.cuda.stream(h2d):
                    x = stage[k][:n].to(dev, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(h2d)
                landed[k] = ev
                compute.wait_event(ev)
                x.record_stream(compute)
                with torch.inference_mode():
                    res = fn.predict_tensors(x)
                for name, t in res.items():
                    outs.setdefault(name, []).append(t)
            out = {name: torch.cat(ts).cpu().numpy() for name, ts in outs.items()}
        return out

    def _map_device_replicas(self, reps, batch_size: int) -> "Dataset":
        import threading

        k = len(reps)
        bounds = [self._n * i // k for i in range(k + 1)]
        parts: list = [None] * k
        errs: list = []

        def run(i):
            try:
                parts[i] = self._map_device(reps[i], batch_size, bounds[i], bounds[i + 1])
            except BaseException as e:  # surfaced below
                errs.append(e)

        ts = [threading.Thread(target=run, args=(i,)) for i in range(k)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errs:
            raise errs[0]
        keys = list(parts[0])
        return Dataset({name: np.concatenate([p[name] for p in parts]) for name in keys})

    def map(self, fn: Callable) -> "Dataset":
        rows = [fn(r) for r in self.take_all()]
        return from_items(rows)

    def limit(self, n: int) -> "Dataset":
        return Dataset({k: v[:n] for k, v in self._cols.items()})

    def __repr__(self):
        return f"Dataset(num_rows={self._n}, schema={self.columns()})"


def from_items(items) -> Dataset:
    """list of row dicts, or a dict of columns."""
    if isinstance(items, dict):
        return Dataset({k: np.asarray(v) for k, v in items.items()})
    if not items:
        return Dataset({})
    keys = list(items[0])
    return Dataset({k: np.stack([np.asarray(r[k]) for r in items]) for k in keys})


def from_numpy(arrs: dict) -> Dataset:
    return Dataset(dict(arrs))


def _is_device_predictor(fn) -> bool:
    dev = getattr(fn, "device", None)
    return hasattr(fn, "predict_tensors") and dev is not None and str(dev).startswith("cuda")


def _gpu_count() -> int:
    try:
        import torch

        return torch.cuda.device_count() if torch.cuda.is_available() else 0
    except Exception:
        return 0


def _accepts_device(cls) -> bool:
    import inspect

    try:
        return "device" in inspect.signature(cls).parameters
    except (TypeError, ValueError):
        return False
