"""Trainer API (the Ray Train surface the reference uses, R/my_ray_module.py:16-25,115-251)."""
from .checkpoint import Checkpoint  # noqa: F401
from .config import CheckpointConfig, FailureConfig, RunConfig, ScalingConfig, TorchConfig  # noqa: F401
from .result import Result  # noqa: F401
from .session import TrainContext, get_checkpoint, get_context, report, report_progress  # noqa: F401
from .trainer import TorchTrainer, TrainingFailedError  # noqa: F401
from . import torch  # noqa: F401,E402
