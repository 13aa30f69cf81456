"""Local run registry + client (the Metaflow datastore/client surface the reference uses:
`Run("RayTorchTrain/<id>").data.result`, `Task("Flow/run/step/task").data.result`,
`current.trigger.run.data.result` - R/train_flow.py:68-73, R/eval_flow.py:42-49).

Layout under RTDC_HOME (default `<cwd>/.rtdc`, like Metaflow's local `.metaflow`):

    <home>/<Flow>/<run_id>/_run.json                      status, params, timestamps
    <home>/<Flow>/<run_id>/<step>/<task_id>/artifacts.json typed JSON artifacts
    <home>/<Flow>/<run_id>/<step>/<task_id>/<name>.parquet|.npy   large artifacts
    <home>/<Flow>/<run_id>/<step>/<task_id>/cards/<id>.html
    <home>/_deployments.json                              deployed flows (schedule/triggers)

Artifacts are never pickled: Results/Checkpoints are JSON, DataFrames parquet, arrays npy
(loaded with allow_pickle=False), so resolving `--from-run` executes nothing from disk.
"""
from __future__ import annotations

import json
import os
import time
from typing import Any

import numpy as np


def home() -> str:
    return os.path.abspath(os.environ.get("RTDC_HOME", os.path.join(os.getcwd(), ".rtdc")))


def run_dir(flow: str, run_id: str) -> str:
    return os.path.join(home(), flow, str(run_id))


def task_dir(flow: str, run_id: str, step: str, task_id: str) -> str:
    return os.path.join(run_dir(flow, run_id), step, str(task_id))


def new_run_id(flow: str) -> str:
    d = os.path.join(home(), flow)
    os.makedirs(d, exist_ok=True)
    n = 1 + max([int(x) for x in os.listdir(d) if x.isdigit()] + [0])
    while True:
        try:
            os.makedirs(os.path.join(d, str(n)))
            return str(n)
        except FileExistsError:
            n += 1


# ------------------------------------------------------------------------------ artifacts
def _encode(name: str, v: Any, tdir: str):
    from ..train.checkpoint import Checkpoint
    from ..train.result import Result

    if isinstance(v, Result):
        return {"__type__": "Result", "value": v.to_json()}
    if isinstance(v, Checkpoint):
        return {"__type__": "Checkpoint", "path": v.path}
    try:
        import pandas as pd

        if isinstance(v, pd.DataFrame):
            fn = f"{name}.parquet"
            df = v.copy()
            for c in df.columns:
                if df[c].dtype == object and len(df) and isinstance(df[c].iloc[0], np.ndarray):
                    df[c] = df[c].apply(lambda a: np.asarray(a).ravel().tolist())
            df.to_parquet(os.path.join(tdir, fn))
            return {"__type__": "DataFrame", "file": fn}
    except ImportError:  # pragma: no cover
        pass
    if isinstance(v, np.ndarray):
        fn = f"{name}.npy"
        np.save(os.path.join(tdir, fn), v, allow_pickle=False)
        return {"__type__": "ndarray", "file": fn}
    try:
        json.dumps(v)
        return v
    except TypeError:
        return {"__type__": "repr", "value": repr(v)}


def _decode(v: Any, tdir: str):
    if isinstance(v, dict) and "__type__" in v:
        t = v["__type__"]
        if t == "Result":
            from ..train.result import Result

            return Result.from_json(v["value"])
        if t == "Checkpoint":
            from ..train.checkpoint import Checkpoint

            return Checkpoint(v["path"])
        if t == "DataFrame":
            import pandas as pd

            return pd.read_parquet(os.path.join(tdir, v["file"]))
        if t == "ndarray":
            return np.load(os.path.join(tdir, v["file"]), allow_pickle=False)
        if t == "repr":
            return v["value"]
    return v


def save_artifacts(tdir: str, artifacts: dict) -> None:
    os.makedirs(tdir, exist_ok=True)
    enc = {k: _encode(k, v, tdir) for k, v in artifacts.items()}
    tmp = os.path.join(tdir, "artifacts.json.tmp")
    with open(tmp, "w") as f:
        json.dump(enc, f, default=str)
    os.replace(tmp, os.path.join(tdir, "artifacts.json"))


def load_artifacts(tdir: str) -> dict:
    p = os.path.join(tdir, "artifacts.json")
    if not os.path.exists(p):
        return {}
    with open(p) as f:
        raw = json.load(f)
    return {k: _decode(v, tdir) for k, v in raw.items()}


def write_run_meta(flow: str, run_id: str, **kw) -> None:
    p = os.path.join(run_dir(flow, run_id), "_run.json")
    meta = {}
    if os.path.exists(p):
        with open(p) as f:
            meta = json.load(f)
    meta.update(kw)
    with open(p + ".tmp", "w") as f:
        json.dump(meta, f, default=str)
    os.replace(p + ".tmp", p)


def read_run_meta(flow: str, run_id: str) -> dict:
    p = os.path.join(run_dir(flow, run_id), "_run.json")
    if not os.path.exists(p):
        return {}
    with open(p) as f:
        return json.load(f)


# ------------------------------------------------------------------------------ client
class _Data:
    def __init__(self, artifacts: dict):
        self.__dict__.update(artifacts)

    def __getattr__(self, k):
        raise AttributeError(f"artifact {k!r} not found")


class Task:
    """`Task("Flow/run_id/step/task_id")`."""

    def __init__(self, pathspec: str):
        parts = pathspec.strip("/").split("/")
        if len(parts) != 4:
            raise ValueError(f"task pathspec must be Flow/run_id/step/task_id, got {pathspec!r}")
        self.flow, self.run_id, self.step, self.id = parts
        self.pathspec = pathspec
        self._dir = task_dir(*parts)
        if not os.path.isdir(self._dir):
            raise KeyError(f"no such task: {pathspec} (registry {home()})")

    @property
    def data(self) -> _Data:
        return _Data(load_artifacts(self._dir))

    @property
    def successful(self) -> bool:
        return os.path.exists(os.path.join(self._dir, "artifacts.json"))

    def __repr__(self):
        return f"Task('{self.pathspec}')"


class Step:
    def __init__(self, flow, run_id, name):
        self.flow, self.run_id, self.name = flow, run_id, name
        self._dir = os.path.join(run_dir(flow, run_id), name)

    def tasks(self):
        if not os.path.isdir(self._dir):
            return []
        return [Task(f"{self.flow}/{self.run_id}/{self.name}/{t}") for t in sorted(os.listdir(self._dir))
                if os.path.isdir(os.path.join(self._dir, t))]

    @property
    def task(self):
        ts = self.tasks()
        return ts[0] if ts else None


class Run:
    """`Run("Flow/run_id")`; `.data` = artifacts of the `end` step (Metaflow semantics)."""

    def __init__(self, pathspec: str):
        parts = pathspec.strip("/").split("/")
        if len(parts) != 2:
            raise ValueError(f"run pathspec must be Flow/run_id, got {pathspec!r}")
        self.flow, self.id = parts
        self.pathspec = pathspec
        self._dir = run_dir(*parts)
        if not os.path.isdir(self._dir):
            raise KeyError(f"no such run: {pathspec} (registry {home()})")

    @property
    def meta(self) -> dict:
        return read_run_meta(self.flow, self.id)

    @property
    def successful(self) -> bool:
        return self.meta.get("status") == "succeeded"

    @property
    def finished(self) -> bool:
        return self.meta.get("status") in ("succeeded", "failed")

    def __getitem__(self, step: str) -> Step:
        return Step(self.flow, self.id, step)

    def steps(self):
        return [Step(self.flow, self.id, s) for s in sorted(os.listdir(self._dir))
                if os.path.isdir(os.path.join(self._dir, s))]

    @property
    def data(self) -> _Data:
        for step in ("end",) + tuple(s.name for s in reversed(self.steps())):
            st = Step(self.flow, self.id, step)
            if st.task is not None and st.task.successful:
                return st.task.data
        return _Data({})

    def __repr__(self):
        return f"Run('{self.pathspec}')"


class Flow:
    def __init__(self, name: str):
        self.name = name

    def runs(self):
        d = os.path.join(home(), self.name)
        if not os.path.isdir(d):
            return []
        ids = sorted([x for x in os.listdir(d) if x.isdigit()], key=int, reverse=True)
        return [Run(f"{self.name}/{i}") for i in ids]

    @property
    def latest_run(self):
        r = self.runs()
        return r[0] if r else None

    @property
    def latest_successful_run(self):
        for r in self.runs():
            if r.successful:
                return r
        return None


def namespace(ns=None):  # Metaflow client API compatibility; local registry has one namespace
    return ns


# ------------------------------------------------------------------------------ deployments
def _dep_path():
    return os.path.join(home(), "_deployments.json")


def load_deployments() -> dict:
    p = _dep_path()
    if not os.path.exists(p):
        return {}
    with open(p) as f:
        return json.load(f)


def save_deployment(flow: str, info: dict) -> None:
    os.makedirs(home(), exist_ok=True)
    d = load_deployments()
    d[flow] = dict(info, deployed_at=time.time())
    with open(_dep_path() + ".tmp", "w") as f:
        json.dump(d, f, indent=1)
    os.replace(_dep_path() + ".tmp", _dep_path())
