"""On-disk layout, checkpoint commit and retention (Ray 2.39 layout):

    <storage_path>/                                   RunConfig(storage_path)  (R/my_ray_module.py:237)
      <experiment>/            TorchTrainer_<YYYY-MM-DD_HH-MM-SS>  (RunConfig.name unset)
        experiment_state.json
        <trial>/               TorchTrainer_<trialid>_00000_0_<date>  == Result.path
          params.json  result.json  progress.csv
          checkpoint_000000/   <- committed checkpoints (num_to_keep newest / best survive)
          checkpoint_000001/

A checkpoint is visible only after commit: files are gathered in `checkpoint_NNNNNN.tmp/`
and rank 0 renames the directory atomically (then fsyncs the trial dir), so a crash never
leaves a half-written `checkpoint_NNNNNN/` (the reference's per-rank same-name overwrite
race, SURVEY §5.2, cannot occur: rank 0's copy of a shared file name wins deterministically).
"""
from __future__ import annotations

import csv
import json
import math
import os
import random
import re
import shutil
import string
import time
from datetime import datetime

CKPT_FMT = "checkpoint_{:06d}"


def new_experiment_name(prefix: str = "TorchTrainer") -> str:
    return f"{prefix}_{datetime.now().strftime('%Y-%m-%d_%H-%M-%S')}"


def new_trial_dirname(prefix: str = "TorchTrainer") -> str:
    tid = "".join(random.choice("0123456789abcdef") for _ in range(5))
    return f"{prefix}_{tid}_00000_0_{datetime.now().strftime('%Y-%m-%d_%H-%M-%S')}"


def fsync_dir(path: str) -> None:
    try:
        fd = os.open(path, os.O_RDONLY)
        try:
            os.fsync(fd)
        finally:
            os.close(fd)
    except OSError:
        pass


def staging_dir(trial_dir: str, index: int) -> str:
    return os.path.join(trial_dir, CKPT_FMT.format(index) + ".tmp")


def final_dir(trial_dir: str, index: int) -> str:
    return os.path.join(trial_dir, CKPT_FMT.format(index))


def merge_into(src: str, dst: str, overwrite: bool) -> None:
    """Copy files of a worker's checkpoint dir into the staging dir (atomic per file)."""
    os.makedirs(dst, exist_ok=True)
    if os.path.abspath(src) == os.path.abspath(dst):
        return
    for root, dirs, files in os.walk(src):
        rel = os.path.relpath(root, src)
        tdir = os.path.join(dst, rel) if rel != "." else dst
        os.makedirs(tdir, exist_ok=True)
        for name in files:
            s = os.path.join(root, name)
            d = os.path.join(tdir, name)
            if os.path.exists(d) and not overwrite:
                continue
            tmp = d + f".part{os.getpid()}"
            shutil.copyfile(s, tmp)
            os.replace(tmp, d)


_RENAME_EXCHANGE = 2


def _exchange(a: str, b: str) -> bool:
    """renameat2(RENAME_EXCHANGE): atomically swap two existing paths (Linux >= 3.15)."""
    try:
        import ctypes

        libc = ctypes.CDLL(None, use_errno=True)
        f = libc.renameat2
    except (OSError, AttributeError):
        return False
    AT_FDCWD = -100
    return f(AT_FDCWD, a.encode(), AT_FDCWD, b.encode(), _RENAME_EXCHANGE) == 0


def commit(trial_dir: str, index: int) -> str:
    """Publish `checkpoint_NNNNNN.tmp/` as `checkpoint_NNNNNN/` atomically.  A final directory
    of the same index (only possible after a crash between a commit and the registry update)
    is never deleted first: the new one is swapped in with RENAME_EXCHANGE and only then is
    the old one removed, so `checkpoint_NNNNNN/` always names a complete checkpoint."""
    src, dst = staging_dir(trial_dir, index), final_dir(trial_dir, index)
    if os.path.exists(dst):
        if _exchange(src, dst):
            shutil.rmtree(src, ignore_errors=True)  # src now holds the replaced checkpoint
            fsync_dir(trial_dir)
            return dst
        # no renameat2: move the old one aside (a rename), then publish - still never a
        # moment where dst names a partial directory
        aside = dst + f".replaced.{os.getpid()}"
        os.replace(dst, aside)
        os.replace(src, dst)
        shutil.rmtree(aside, ignore_errors=True)
    else:
        os.replace(src, dst)
    fsync_dir(trial_dir)
    return dst


def sweep_stale_staging(trial_dir: str) -> list[str]:
    """Remove what a crashed attempt left behind: `checkpoint_*.tmp/` staging directories
    (partial shards of a checkpoint that was never committed) and `*.replaced.*` leftovers.
    Called by the driver before every attempt, while no worker runs, so a restarted attempt
    never commits a staging dir that still holds a dead attempt's partial files."""
    removed = []
    if not os.path.isdir(trial_dir):
        return removed
    for name in os.listdir(trial_dir):
        if name.startswith("checkpoint_") and (name.endswith(".tmp") or ".replaced." in name):
            p = os.path.join(trial_dir, name)
            shutil.rmtree(p, ignore_errors=True)
            removed.append(p)
    if removed:
        fsync_dir(trial_dir)
    return removed


def list_committed(trial_dir: str) -> list[tuple[int, str]]:
    out = []
    if not os.path.isdir(trial_dir):
        return out
    for name in os.listdir(trial_dir):
        if name.startswith("checkpoint_") and not name.endswith(".tmp") and name[11:].isdigit():
            out.append((int(name[11:]), os.path.join(trial_dir, name)))
    return sorted(out)


def latest_committed(trial_dir: str) -> str | None:
    c = list_committed(trial_dir)
    return c[-1][1] if c else None


REGISTRY_FN = ".checkpoints.json"


class TrialLogger:
    """result.json (JSON lines) + progress.csv + checkpoint registry with retention (rank 0)."""

    def __init__(self, trial_dir: str, num_to_keep=None, score_attr=None, score_order="max"):
        self.trial_dir = trial_dir
        self.num_to_keep = num_to_keep
        self.score_attr = score_attr
        self.score_order = score_order
        self.t0 = time.time()
        self.iteration = 0
        self.kept: list[tuple[int, str, dict]] = []  # (index, path, metrics)
        self._csv_fields = None
        reg = os.path.join(trial_dir, REGISTRY_FN)
        if os.path.exists(reg):
            try:
                with open(reg) as f:
                    self.kept = [tuple(x) for x in json.load(f)]
            except (ValueError, TypeError, OSError):
                # unreadable registry (a crash of an older writer, a damaged disk): rebuild it
                # from the committed checkpoint directories - the directories, not the registry,
                # are the commit record (storage.commit renames them into place atomically)
                self.kept = self._scan_committed()
                self._write_registry()
            self.iteration = max([m.get("training_iteration", 0) for _, _, m in self.kept] + [0])

    def log(self, metrics: dict, checkpoint_index: int | None) -> dict:
        self.iteration += 1
        now = time.time()
        row = dict(metrics)
        row.update({
            "timestamp": int(now),
            "checkpoint_dir_name": CKPT_FMT.format(checkpoint_index) if checkpoint_index is not None else None,
            "done": False,
            "training_iteration": self.iteration,
            "time_total_s": now - self.t0,
            "date": datetime.now().strftime("%Y-%m-%d_%H-%M-%S"),
            "pid": os.getpid(),
        })
        with open(os.path.join(self.trial_dir, "result.json"), "a") as f:
            f.write(json.dumps(row, default=str) + "\n")
        csv_path = os.path.join(self.trial_dir, "progress.csv")
        flat = {k: v for k, v in row.items() if not isinstance(v, (dict, list))}
        new = not os.path.exists(csv_path)
        if self._csv_fields is None:
            self._csv_fields = list(flat.keys())
        with open(csv_path, "a", newline="") as f:
            w = csv.DictWriter(f, fieldnames=self._csv_fields, extrasaction="ignore")
            if new:
                w.writeheader()
            w.writerow(flat)
        return row

    def _score(self, m: dict):
        v = m.get(self.score_attr)
        if v is None or (isinstance(v, float) and math.isnan(v)):
            return -math.inf if self.score_order == "max" else math.inf
        return v

    def register(self, index: int, path: str, metrics: dict) -> list[str]:
        """Record a committed checkpoint; delete what retention drops.  Returns deleted paths."""
        self.kept.append((index, path, metrics))
        deleted = []
        if self.num_to_keep is not None and len(self.kept) > self.num_to_keep:
            if self.score_attr:
                rev = self.score_order == "max"
                ranked = sorted(self.kept, key=lambda x: self._score(x[2]), reverse=rev)
                keep = ranked[: self.num_to_keep]
                # never delete the most recent checkpoint (needed for fault-tolerant resume)
                latest = max(self.kept, key=lambda x: x[0])
                if latest not in keep:
                    keep = keep[:-1] + [latest]
            else:
                keep = sorted(self.kept, key=lambda x: x[0])[-self.num_to_keep:]
            keep_idx = {k[0] for k in keep}
            for k in self.kept:
                if k[0] not in keep_idx:
                    shutil.rmtree(k[1], ignore_errors=True)
                    deleted.append(k[1])
            self.kept = sorted(keep, key=lambda x: x[0])
        self._write_registry()
        return deleted

    def _write_registry(self) -> None:
        """tmp + fsync + rename: a crash leaves the old or the new registry, never a torn one."""
        reg = os.path.join(self.trial_dir, REGISTRY_FN)
        tmp = f"{reg}.tmp.{os.getpid()}"
        with open(tmp, "w") as f:
            json.dump([list(k) for k in self.kept], f, default=str)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, reg)
        fsync_dir(self.trial_dir)

    def _scan_committed(self) -> list:
        """(index, path, metrics) of every committed checkpoint directory, metrics from result.json."""
        rows = {}
        try:
            with open(os.path.join(self.trial_dir, "result.json")) as f:
                for line in f:
                    try:
                        r = json.loads(line)
                    except ValueError:
                        continue  # a torn last line
                    if r.get("checkpoint_dir_name"):
                        rows[r["checkpoint_dir_name"]] = r
        except OSError:
            pass
        out = []
        for name in sorted(os.listdir(self.trial_dir)):
            m = re.fullmatch(r"checkpoint_(\d{6})", name)
            if m and os.path.isdir(os.path.join(self.trial_dir, name)):
                out.append((int(m.group(1)), os.path.join(self.trial_dir, name), rows.get(name, {})))
        return out

    def best_checkpoints(self):
        return list(self.kept)
