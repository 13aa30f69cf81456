"""`Checkpoint`: a handle to a directory of checkpoint files (Ray Train semantics).

Reference usage: `Checkpoint.from_directory(tmpdir)` on every rank before `report`
(R/my_ray_module.py:202), `checkpoint.as_directory()` on restore (:254), `checkpoint.path`
(:133), `Result.checkpoint` (R/train_flow.py:70,73).  Local filesystem only; the handle is
a plain path (picklable, JSON-serialisable) so runs can be resumed from the run registry.
"""
from __future__ import annotations

import contextlib
import json
import os
import shutil
import tempfile

_META = ".metadata.json"


class Checkpoint:
    def __init__(self, path: str, filesystem=None):
        self.path = os.path.abspath(os.fspath(path))
        self.filesystem = filesystem
        self._pending = None  # AsyncSave handle (sharded async checkpoints)

    @classmethod
    def from_directory(cls, path) -> "Checkpoint":
        return cls(path)

    @contextlib.contextmanager
    def as_directory(self):
        """Local path of the checkpoint (already local: yielded as-is, never deleted)."""
        self.wait()
        yield self.path

    def to_directory(self, path: str | None = None) -> str:
        self.wait()
        dst = path or tempfile.mkdtemp(prefix="checkpoint_")
        os.makedirs(dst, exist_ok=True)
        for name in os.listdir(self.path):
            s = os.path.join(self.path, name)
            d = os.path.join(dst, name)
            if os.path.isdir(s):
                shutil.copytree(s, d, dirs_exist_ok=True)
            else:
                shutil.copy2(s, d)
        return dst

    def get_metadata(self) -> dict:
        p = os.path.join(self.path, _META)
        if os.path.exists(p):
            with open(p) as f:
                return json.load(f)
        return {}

    def set_metadata(self, metadata: dict) -> None:
        with open(os.path.join(self.path, _META), "w") as f:
            json.dump(metadata, f)

    def update_metadata(self, metadata: dict) -> None:
        m = self.get_metadata()
        m.update(metadata)
        self.set_metadata(m)

    def wait(self):
        """Block until an asynchronously written checkpoint is durable."""
        if self._pending is not None:
            self._pending.wait()
            self._pending = None
        return self

    def __getstate__(self):
        return {"path": self.path}

    def __setstate__(self, st):
        self.path = st["path"]
        self.filesystem = None
        self._pending = None

    @classmethod
    def from_async_save(cls, handle) -> "Checkpoint":
        """Wrap an in-flight `checkpoint.dcp.async_save` handle; `report()` commits it in the
        background once every rank's shard is durable (rank 0 writes `.metadata`)."""
        c = cls(handle.checkpoint_id)
        c._pending = handle
        c._handle = handle
        return c

    def _finish(self):
        h = getattr(self, "_handle", None)
        if h is not None:
            h._finish()

    def __repr__(self):
        return f"Checkpoint(filesystem=local, path={self.path})"

    def __eq__(self, other):
        return isinstance(other, Checkpoint) and other.path == self.path

    def __hash__(self):
        return hash(self.path)
