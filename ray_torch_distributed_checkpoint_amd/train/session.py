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
engine straight into the staging dir (`get_context().next_checkpoint_dir()`) and a background
committer runs steps 2-3 once every rank's write is durable, so `report` returns immediately;
the driver learns the checkpoint path only after that commit.  The stage / write / commit
seconds of each async checkpoint are attached to the next reported metrics row
(`ckpt_stage_s`, `ckpt_write_s`, `ckpt_commit_s`, `ckpt_index`).

Progress and fault injection: `report_progress(step)` publishes a monotone step
counter from the TRAINING thread (rate-limited TCPStore writes), which the supervisor watches
for stalls - unlike the heartbeat thread, it stops when the training thread is stuck in a
collective.  It is also the step-granular fault-injection point (first attempt only):
  RTDC_FAIL_AT_STEP=K[:rank]  SIGKILL at the start of step K,
  RTDC_HANG_AT_STEP=K[:rank]  block forever at the start of step K (peers then hang in their
                              next collective: a real collective stall).
"""
from __future__ import annotations

import json
import os
import queue
import signal
import threading
import time
from dataclasses import dataclass, field
from typing import Any

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
    torch_config: Any = None
    checkpoint_config: Any = None
    run_config: Any = field(default=None, repr=False)

    def get_torch_config(self):
        from .config import TorchConfig

        return self.torch_config or TorchConfig()

    def get_checkpoint_config(self):
        from .config import CheckpointConfig

        return self.checkpoint_config or CheckpointConfig()

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
        self._ckpt_timing: dict = {}  # timings of the last completed async checkpoint
        self._timing_lock = threading.Lock()
        # progress publishing + fault injection
        self._prog_key = f"a{ctx.attempt}/prog/{ctx.world_rank}"
        self._prog_last = 0.0
        self._prog_step = -1
        self._prog_explicit = False  # set by the first report_progress(): only those ranks are watched
        self._prog_seq = 0           # advanced by every report(), so report-only loops never look stalled
        self._fail_at = self._parse_injector("RTDC_FAIL_AT_STEP")
        self._hang_at = self._parse_injector("RTDC_HANG_AT_STEP")

    def _parse_injector(self, var):
        v = os.environ.get(var)
        if not v or self.ctx.attempt != 0:
            return None
        k, _, r = v.partition(":")
        if r and int(r) != self.ctx.world_rank:
            return None
        return int(k)

    # ------------------------------------------------------------------ progress
    def report_progress(self, step: int, force: bool = False):
        if self._fail_at is not None and step >= self._fail_at:
            os.kill(os.getpid(), signal.SIGKILL)
        if self._hang_at is not None and step >= self._hang_at:
            self._publish_progress(step)
            threading.Event().wait()  # never returns: the gang is killed by the supervisor
        self._prog_step = max(self._prog_step, int(step))
        first = not self._prog_explicit
        self._prog_explicit = True
        now = time.time()
        if force or first or now - self._prog_last >= 1.0:
            self._publish_progress(self._prog_step, now)

    def _publish_progress(self, step, now=None):
        """Publish `<step> <time> <report seq>`; the supervisor treats a change of either the
        step or the report sequence as progress.  Nothing is published for a loop that never
        called `report_progress` (a Ray-style loop that only reports once per epoch must not
        be judged by a per-step timeout)."""
        if not self._prog_explicit:
            return
        now = now or time.time()
        self._prog_last = now
        try:
            self.store.set(self._prog_key, f"{step} {now} {self._prog_seq}")
        except Exception:
            pass

    # ------------------------------------------------------------------ report
    def report(self, metrics: dict, checkpoint: Checkpoint | None = None):
        if self._commit_err:
            raise self._commit_err
        from ..parallel import health

        # a rank whose gradient collective timed out (NaN-poisoned, update skipped) fails here,
        # before the commit barrier: the attempt dies and nothing of this report is committed.
        # With a checkpoint attached, its save decides from the words captured at its snapshot
        # (no device sync on the async path); without one, synchronise so every collective
        # enqueued so far has completed or recorded its timeout
        health.assert_healthy("report", sync=checkpoint is None)
        rank = self.ctx.world_rank
        n = self.n_reports
        key = f"s{self.ctx.attempt}/r{n}"
        stage = storage.staging_dir(self.ctx.trial_dir, self.next_index)
        is_async = checkpoint is not None and (
            checkpoint._pending is not None or os.path.abspath(checkpoint.path) == os.path.abspath(stage))
        if is_async and os.path.abspath(checkpoint.path) != os.path.abspath(stage):
            # an in-place (async) checkpoint must have been written into the directory this
            # report commits; anything else would commit an empty staging dir
            raise ValueError(f"async checkpoint written to {checkpoint.path}, but this report commits {stage}: "
                             f"save into train.get_context().next_checkpoint_dir()")
        self._prog_seq += 1
        self._publish_progress(self._prog_step)
        with self._timing_lock:
            if self._ckpt_timing:
                metrics = dict(metrics, **self._ckpt_timing)
                self._ckpt_timing = {}
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
            # an async checkpoint is announced by the committer once it is committed
            done = idx is not None and not any_async
            self._publish({"type": "report", "metrics": row,
                           "checkpoint": storage.final_dir(self.ctx.trial_dir, idx) if done else None})
        self.barrier.wait(f"r{n}d")
        self.n_reports += 1

    def _publish(self, msg: dict):
        k = self.store.add(f"a{self.ctx.attempt}/nreports", 1)
        self.store.set(f"a{self.ctx.attempt}/report/{k}", json.dumps(msg, default=str))

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
                t_q = time.perf_counter()
                h = getattr(ck, "_handle", None) if ck is not None else None
                if ck is not None:
                    ck.wait()  # this rank's shard files durable
                timing = {"ckpt_index": idx}
                if h is not None and getattr(h, "t_return", None) is not None:
                    timing["ckpt_stage_s"] = round(h.t_return, 6)
                    timing["ckpt_write_s"] = round(h.write_s if h.write_s is not None else 0.0, 6)
                key = f"s{self.ctx.attempt}/commit/{idx}"
                self.store.add(key, 1)
                if self.ctx.world_rank == 0:
                    t0 = time.time()
                    while self.store.add(key, 0) < self.ctx.world_size:
                        if time.time() - t0 > 3600:
                            raise TimeoutError("async checkpoint commit barrier timed out")
                        time.sleep(0.002)
                    t_c = time.perf_counter()
                    if ck is not None and hasattr(ck, "_finish"):
                        ck._finish()  # rank-0 metadata write (DCP .metadata)
                    stage = storage.staging_dir(self.ctx.trial_dir, idx)
                    if not os.path.isdir(stage):
                        raise FileNotFoundError(f"async checkpoint staging dir {stage} missing at commit")
                    path = storage.commit(self.ctx.trial_dir, idx)
                    self.logger.register(idx, path, metrics)
                    timing["ckpt_commit_s"] = round(time.perf_counter() - t_c, 6)
                    timing["ckpt_durable_s"] = round(time.perf_counter() - t_q + timing.get("ckpt_stage_s", 0.0), 6)
                    self.store.set(f"s{self.ctx.attempt}/committed/{idx}", path)
                    self._publish({"type": "commit", "index": idx, "checkpoint": path})
                with self._timing_lock:
                    self._ckpt_timing = timing
            except BaseException as e:  # surfaced on the next report / at shutdown
                self._commit_err = e
            finally:
                self._commit_q.task_done()

    def flush(self):
        """Wait for every queued async checkpoint to be committed."""
        if self._committer is not None:
            self._commit_q.join()
        if self._commit_err:
            raise self._commit_err

    def close(self):
        self.flush()
        if self._committer is not None:
            self._commit_q.put(None)
        try:
            self.store.set(self._prog_key, "done")
        except Exception:
            pass


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


def report_progress(step: int) -> None:
    """Publish the training step counter to the supervisor (stall detection) - cheap enough to
    call every step; also where RTDC_FAIL_AT_STEP / RTDC_HANG_AT_STEP fire.  No-op outside a
    trainer."""
    s = _get_session(required=False)
    if s is not None:
        s.report_progress(step)


def get_checkpoint() -> Checkpoint | None:
    s = _get_session(required=False)
    return None if s is None else s.resume_checkpoint
