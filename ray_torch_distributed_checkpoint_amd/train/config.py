"""Run/scaling/checkpoint/failure configuration (the Ray Train config surface the reference uses).

Reference call sites: `RunConfig(checkpoint_config=CheckpointConfig(num_to_keep=...),
storage_path=..., verbose=1)` and `ScalingConfig(num_workers=..., use_gpu=...)`
(R/my_ray_module.py:235-243).  Field names and defaults follow Ray 2.39; MI355X knobs are
added in the same style (`bucket_cap_mb`, `ckpt_slot_mb`, ...).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Any, Optional


@dataclass
class ScalingConfig:
    num_workers: int = 1
    use_gpu: bool = False
    resources_per_worker: Optional[dict] = None
    placement_strategy: str = "PACK"
    trainer_resources: Optional[dict] = None

    @property
    def num_gpus_per_worker(self) -> int:
        if self.resources_per_worker and "GPU" in self.resources_per_worker:
            return int(self.resources_per_worker["GPU"])
        return 1 if self.use_gpu else 0


@dataclass
class CheckpointConfig:
    num_to_keep: Optional[int] = None
    checkpoint_score_attribute: Optional[str] = None
    checkpoint_score_order: str = "max"
    checkpoint_frequency: int = 0
    checkpoint_at_end: Optional[bool] = None

    def __post_init__(self):
        if self.num_to_keep is not None and self.num_to_keep <= 0:
            raise ValueError("num_to_keep must be a positive integer or None")
        if self.checkpoint_score_order not in ("max", "min"):
            raise ValueError("checkpoint_score_order must be 'max' or 'min'")


@dataclass
class FailureConfig:
    """max_failures: restarts of the whole worker group, each resuming from the latest
    committed checkpoint of the same trial (the reference has only Metaflow @retry, which
    restarts from scratch - SURVEY §5.3)."""
    max_failures: int = 0
    fail_fast: bool = False


@dataclass
class RunConfig:
    name: Optional[str] = None
    storage_path: Optional[str] = None
    checkpoint_config: CheckpointConfig = field(default_factory=CheckpointConfig)
    failure_config: FailureConfig = field(default_factory=FailureConfig)
    verbose: int = 1
    stop: Any = None
    callbacks: Any = None
    log_to_file: bool = False
    # MI355X-native knobs
    worker_timeout_s: float = 1800.0  # process-group timeout (Ray TorchConfig default)
    heartbeat_timeout_s: float = 600.0

    def resolved_storage_path(self) -> str:
        p = self.storage_path or os.environ.get("RTDC_STORAGE_PATH") or os.path.join("~", "rtdc_results")
        return os.path.abspath(os.path.expanduser(str(p)))


@dataclass
class TorchConfig:
    backend: Optional[str] = None  # None -> "nccl" (RCCL) with GPUs, "gloo" on CPU
    init_method: str = "env"
    timeout_s: int = 1800
