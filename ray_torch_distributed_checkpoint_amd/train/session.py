"""Worker-side session: `report`, `get_context`, `get_checkpoint` (Ray Train worker API).

Reference call sites: `ray.train.get_context().get_world_size()/get_world_rank()`
(R/my_ray_module.py:149,177), `ray.train.report({"val_loss","accuracy"}, checkpoint=...)`
(:203-205).

`report` semantics (made race-free):
  1. every rank gathers its checkpoint files into `checkpoint_NNNNNN.tmp/` - rank 0 first
     (its files win a name clash), then the others add only files that do not exist yet;
  2. a control-plane barrier (TCPStore, never the RCCL communicator, so it cannot interleave
     with gradient collectives);
  3. rank 0 renames the directory (atomic commit), appends result.json / progress.csv,
     enforces `num_to_keep`, publishes the metrics to the driver;
  4. barrier - the report call synchronises workers like Ray's.
Asynchronous (sharded DCP) checkpoints skip step 1: shards are written by the native
engine straight into the staging dir and a background committer runs steps 2-3 once every
rank's write is durable, so `report` returns immediately.
"""
from __future__ import annotations

import json
import os
import queue
import threading
import time
from dataclasses import dataclass

from . import storage
from .checkpoint import Checkpoint


class StoreBarrier:
    """Counter barrier on a torch TCPStore (control plane only)."""

    def __init__(self, store, world_size: int, prefix: str):
        self.store, self.world, self.prefix = store, world_size, prefix
        self.n = 0

    def wait(self, name: str | None = None, timeout_s: float = 1800.0):
        self.n += 1
        key = f"{self.prefix}/bar/{name or self.n}"
        self.store.add(key, 1)
        t0 = time.time()
        delay = 0.0005
        while self.store.add(key, 0) < self.world:
            if time.time() - t0 > timeout_s:
                raise TimeoutError(f"store barrier {key} timed out")
            time.sleep(delay)
            delay = min(delay * 2, 0.05)


@dataclass
class TrainContext:
    world_size: int
    world_rank: int
    local_rank: int
    local_world_size: int
    node_rank: int
    experiment_name: str
    trial_dir: str
    storage_path: str
    trial_name: str
    attempt: int = 0

    def get_world_size(self):
        return self.world_size

    def get_world_rank(self):
        return self.world_rank

    def get_local_rank(self):
        return self.local_rank

    def get_local_world_size(self):
        return self.local_world_size

    def get_node_rank(self):
        return self.node_rank

    def get_experiment_name(self):
        return self.experiment_name

    def get_trial_name(self):
        return self.trial_name

    def get_trial_dir(self):
        return self.trial_dir

    def get_storage(self):
        return self.storage_path

    def next_checkpoint_dir(self) -> str:
        """Staging directory the NEXT `report` commits (for shards written in place)."""
        s = _session
        idx = s.next_index if s else 0
        d = storage.staging_dir(self.trial_dir, idx)
        os.makedirs(d, exist_ok=True)
        return d


class _Session:
    def __init__(self, ctx: TrainContext, store, ckpt_cfg, resume_checkpoint: Checkpoint | None):
        self.ctx = ctx
        self.store = store
        self.barrier = StoreBarrier(store, ctx.world_size, f"s{ctx.attempt}")
        self.resume_checkpoint = resume_checkpoint
        existing = storage.list_committed(ctx.trial_dir)
        self.next_index = (existing[-1][0] + 1) if existing else 0
        self.logger = None
        if ctx.world_rank == 0:
            self.logger = storage.TrialLogger(ctx.trial_dir, ckpt_cfg.num_to_keep,
                                              ckpt_cfg.checkpoint_score_attribute, ckpt_cfg.checkpoint_score_order)
        self.n_reports = 0
        self._commit_q: queue.Queue = queue.Queue()
        self._committer = None
        self._commit_err = None
        self.last_metrics = None

    # ------------------------------------------------------------------ report
    def report(self, metrics: dict, checkpoint: Checkpoint | None = None):
        if self._commit_err:
            raise self._commit_err
        rank = self.ctx.world_rank
        n = self.n_reports
        key = f"s{self.ctx.attempt}/r{n}"
        stage = storage.staging_dir(self.ctx.trial_dir, self.next_index)
        is_async = checkpoint is not None and (
            checkpoint._pending is not None or os.path.abspath(checkpoint.path) == os.path.abspath(stage))
        if checkpoint is not None:
            self.store.add(key + "/ck", 1)
        if is_async:
            self.store.add(key + "/async", 1)
        self.barrier.wait(f"r{n}a")
        any_ck = self.store.add(key + "/ck", 0) > 0
        any_async = self.store.add(key + "/async", 0) > 0
        idx = None
        if any_ck:
            idx = self.next_index
            self.next_index += 1
            if any_async:
                # async / in-place shards: commit in the background once every rank is durable
                self._enqueue_commit(idx, checkpoint, metrics)
            else:
                if rank == 0 and checkpoint is not None:
                    storage.merge_into(checkpoint.path, stage, overwrite=True)
                self.barrier.wait(f"r{n}b")
                if rank != 0 and checkpoint is not None:
                    storage.merge_into(checkpoint.path, stage, overwrite=False)
                self.barrier.wait(f"r{n}c")
                if rank == 0:
                    os.makedirs(stage, exist_ok=True)
                    path = storage.commit(self.ctx.trial_dir, idx)
                    self.logger.register(idx, path, dict(metrics))
        row = None
        if rank == 0:
            row = self.logger.log(metrics, idx)
            self.last_metrics = row
            self._publish(row, None if idx is None else storage.final_dir(self.ctx.trial_dir, idx))
        self.barrier.wait(f"r{n}d")
        self.n_reports += 1

    def _publish(self, row, ckpt_path):
        msg = json.dumps({"metrics": row, "checkpoint": ckpt_path}, default=str)
        k = self.store.add(f"a{self.ctx.attempt}/nreports", 1)
        self.store.set(f"a{self.ctx.attempt}/report/{k}", msg)

    # ------------------------------------------------------------------ async commits
    def _enqueue_commit(self, idx, checkpoint, metrics):
        if self._committer is None:
            self._committer = threading.Thread(target=self._commit_loop, daemon=True)
            self._committer.start()
        self._commit_q.put((idx, checkpoint, dict(metrics)))

    def _commit_loop(self):
        while True:
            item = self._commit_q.get()
            if item is None:
                return
            idx, ck, metrics = item
            try:
                if ck is not None:
                    ck.wait()  # this rank's shard files durable
                key = f"s{self.ctx.attempt}/commit/{idx}"
                self.store.add(key, 1)
                if self.ctx.world_rank == 0:
                    t0 = time.time()
                    while self.store.add(key, 0) < self.ctx.world_size:
                        if time.time() - t0 > 3600:
                            raise TimeoutError("async checkpoint commit barrier timed out")
                        time.sleep(0.002)
                    if ck is not None and hasattr(ck, "_finish"):
                        ck._finish()  # rank-0 metadata write (DCP .metadata)
                    os.makedirs(storage.staging_dir(self.ctx.trial_dir, idx), exist_ok=True)
                    path = storage.commit(self.ctx.trial_dir, idx)
                    self.logger.register(idx, path, metrics)
                    self.store.set(f"s{self.ctx.attempt}/committed/{idx}", path)
            except BaseException as e:  # surfaced on the next report / at shutdown
                self._commit_err = e
            finally:
                self._commit_q.task_done()

    def flush(self):
        """Wait for every queued async checkpoint to be committed."""
        if self._committer is not None:
            self._commit_q.join()
            if self.ctx.world_rank == 0:
                pass
        if self._commit_err:
            raise self._commit_err

    def close(self):
        self.flush()
        if self._committer is not None:
            self._commit_q.put(None)


_session: _Session | None = None


def _set_session(s):
    global _session
    _session = s


def _get_session(required=True) -> _Session | None:
    if _session is None and required:
        raise RuntimeError("not inside a training worker (call from train_loop_per_worker)")
    return _session


def report(metrics: dict, checkpoint: Checkpoint | None = None) -> None:
    _get_session().report(metrics, checkpoint)


def get_context() -> TrainContext:
    s = _get_session(required=False)
    if s is None:
        # outside a trainer (e.g. torchrun): derive from env
        ws = int(os.environ.get("WORLD_SIZE", "1"))
        return TrainContext(ws, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
                            int(os.environ.get("LOCAL_WORLD_SIZE", str(ws))), int(os.environ.get("NODE_RANK", "0")),
                            "", "", "", "")
    return s.ctx


def get_checkpoint() -> Checkpoint | None:
    s = _get_session(required=False)
    return None if s is None else s.resume_checkpoint
