"""`TorchTrainer(...).fit() -> Result` (the Ray Train driver the reference calls at
R/my_ray_module.py:244-250), on the process-per-GPU launcher.

fit():
  1. resolve the storage layout (`<storage_path>/<experiment>/<trial>/`, RunConfig semantics);
  2. ship `train_loop_per_worker` + `train_loop_config` (cloudpickle, like Ray) to
     `ScalingConfig.num_workers` worker processes;
  3. supervise the gang; on a failure restart (FailureConfig.max_failures) from the latest
     committed checkpoint of the trial;
  4. return a `Result` (last rank-0 metrics, latest committed checkpoint, trial path,
     error, retained checkpoints).
"""
from __future__ import annotations

import json
import os
import shutil

from . import storage
from .checkpoint import Checkpoint
from .config import CheckpointConfig, FailureConfig, RunConfig, ScalingConfig, TorchConfig
from .launcher import WorkerGroup, write_payload
from .result import Result


class TrainingFailedError(RuntimeError):
    pass


class TorchTrainer:
    def __init__(self, train_loop_per_worker, *, train_loop_config: dict | None = None,
                 scaling_config: ScalingConfig | None = None, run_config: RunConfig | None = None,
                 torch_config: TorchConfig | None = None, resume_from_checkpoint: Checkpoint | None = None,
                 datasets=None, metadata=None):
        self.fn = train_loop_per_worker
        self.config = train_loop_config or {}
        self.scaling = scaling_config or ScalingConfig()
        self.run = run_config or RunConfig()
        self.torch_config = torch_config or TorchConfig()
        self.resume = resume_from_checkpoint
        self.datasets = datasets
        self.metadata = metadata

    def fit(self) -> Result:
        root = self.run.resolved_storage_path()
        exp = self.run.name or storage.new_experiment_name()
        exp_dir = os.path.join(root, exp)
        trial = storage.new_trial_dirname()
        trial_dir = os.path.join(exp_dir, trial)
        os.makedirs(trial_dir, exist_ok=True)
        with open(os.path.join(exp_dir, "experiment_state.json"), "w") as f:
            json.dump({"trial": trial, "num_workers": self.scaling.num_workers, "use_gpu": self.scaling.use_gpu}, f)
        with open(os.path.join(trial_dir, "params.json"), "w") as f:
            json.dump({"train_loop_config": self.config}, f, default=repr)
        ck_cfg = self.run.checkpoint_config or CheckpointConfig()
        fail_cfg = self.run.failure_config or FailureConfig()
        n = self.scaling.num_workers
        if self.scaling.use_gpu:
            import torch

            avail = torch.cuda.device_count()
            if avail < n:
                raise RuntimeError(f"ScalingConfig asks for {n} GPU workers but only {avail} GPUs are visible")
        group = WorkerGroup(n, self.scaling.use_gpu, self.run.verbose)
        resume = self.resume.path if self.resume is not None else None
        last = {"metrics": None, "checkpoint": None}
        errors = []

        def on_report(msg):
            if msg.get("checkpoint"):
                last["checkpoint"] = msg["checkpoint"]
            if msg.get("type") == "commit":
                if self.run.verbose:
                    print(f"[rtdc] committed {msg['checkpoint']}", flush=True)
                return
            last["metrics"] = msg["metrics"]
            if self.run.verbose:
                m = {k: v for k, v in msg["metrics"].items()
                     if k in ("training_iteration", "step", "val_loss", "accuracy", "loss", "samples_per_s",
                              "time_total_s")}
                print(f"[rtdc] report {m}", flush=True)

        attempts = fail_cfg.max_failures + 1 if fail_cfg.max_failures >= 0 else 10 ** 9
        attempt = 0
        outcome = None
        while attempt < attempts:
            payload = {
                "fn": self.fn, "config": self.config, "use_gpu": self.scaling.use_gpu,
                "backend": self.torch_config.backend, "timeout_s": self.torch_config.timeout_s,
                "experiment_name": exp, "trial_dir": trial_dir, "storage_path": root,
                "checkpoint_config": ck_cfg, "resume_checkpoint": resume, "torch_config": self.torch_config,
            }
            ppath = write_payload(payload)
            stale = storage.sweep_stale_staging(trial_dir)  # a failed attempt's partial shards
            if stale and self.run.verbose:
                print(f"[rtdc] removed {len(stale)} uncommitted staging dir(s) of a failed attempt", flush=True)
            try:
                group.start(ppath, attempt)
                outcome = group.supervise(attempt, self.run.heartbeat_timeout_s, on_report,
                                          self.run.progress_timeout_s)
            finally:
                shutil.rmtree(os.path.dirname(ppath), ignore_errors=True)
            if outcome.ok:
                break
            errors.append(outcome.error)
            if self.run.verbose:
                print(f"[rtdc] worker group failed (attempt {attempt}): {outcome.error.splitlines()[-1] if outcome.error else ''}",
                      flush=True)
            if fail_cfg.fail_fast:
                break
            attempt += 1
            # restart from the latest committed checkpoint of this trial (if any)
            latest = storage.latest_committed(trial_dir)
            if latest is not None:
                resume = latest
        committed = storage.latest_committed(trial_dir)
        ckpt = Checkpoint(committed) if committed else None
        kept = []
        reg = os.path.join(trial_dir, ".checkpoints.json")
        if os.path.exists(reg):
            with open(reg) as f:
                kept = [(Checkpoint(p), m) for _, p, m in json.load(f) if os.path.exists(p)]
        res = Result(metrics=last["metrics"], checkpoint=ckpt, path=trial_dir, best_checkpoints=kept)
        if outcome is None or not outcome.ok:
            msg = "\n".join(e for e in errors if e)
            res.error = TrainingFailedError(msg or "training failed")
            res._error_text = msg
            raise res.error
        return res
