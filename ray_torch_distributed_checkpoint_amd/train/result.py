"""`Result` of `TorchTrainer.fit()` (Ray 2.39 `ray.train.Result` surface used by the reference:
`.checkpoint` (R/train_flow.py:70,73; R/eval_flow.py:42-49), `.metrics`, `.path`, `.error`).

Serialised as JSON (never pickle) into the run registry, so a later `--from-run` resolves
the checkpoint without unpickling anything.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from typing import Any, Optional

from .checkpoint import Checkpoint


@dataclass
class Result:
    metrics: Optional[dict] = None
    checkpoint: Optional[Checkpoint] = None
    error: Optional[BaseException] = None
    path: Optional[str] = None
    best_checkpoints: list = field(default_factory=list)  # [(Checkpoint, metrics)]
    _error_text: Optional[str] = None

    @property
    def metrics_dataframe(self):
        import pandas as pd

        if not self.path:
            return None
        p = os.path.join(self.path, "progress.csv")
        return pd.read_csv(p) if os.path.exists(p) else None

    @property
    def config(self) -> Any:
        if self.path and os.path.exists(os.path.join(self.path, "params.json")):
            with open(os.path.join(self.path, "params.json")) as f:
                return json.load(f)
        return None

    def get_best_checkpoint(self, metric: str, mode: str = "max") -> Optional[Checkpoint]:
        cands = [(c, m) for c, m in self.best_checkpoints if metric in m]
        if not cands:
            return None
        key = (lambda cm: cm[1][metric])
        return (max if mode == "max" else min)(cands, key=key)[0]

    def to_json(self) -> dict:
        return {
            "metrics": self.metrics,
            "checkpoint": None if self.checkpoint is None else self.checkpoint.path,
            "path": self.path,
            "error": None if self.error is None and not self._error_text else (self._error_text or repr(self.error)),
            "best_checkpoints": [(c.path, m) for c, m in self.best_checkpoints],
        }

    @classmethod
    def from_json(cls, d: dict) -> "Result":
        r = cls(metrics=d.get("metrics"), checkpoint=Checkpoint(d["checkpoint"]) if d.get("checkpoint") else None,
                path=d.get("path"), best_checkpoints=[(Checkpoint(p), m) for p, m in d.get("best_checkpoints", [])])
        r._error_text = d.get("error")
        if r._error_text:
            r.error = RuntimeError(r._error_text)
        return r

    def __repr__(self):
        shown = {k: v for k, v in (self.metrics or {}).items() if k in ("val_loss", "accuracy", "training_iteration")}
        return f"Result(metrics={shown}, path='{self.path}', filesystem='local', checkpoint={self.checkpoint})"
