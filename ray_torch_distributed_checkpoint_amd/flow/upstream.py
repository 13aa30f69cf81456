"""Upstream-checkpoint resolution shared by train_flow.py (warm start) and eval_flow.py.

Precedence (R/eval_flow.py:40-54, R/train_flow.py:65-72): the run that triggered this one (eval
only), then an explicit task pathspec, then an explicit run pathspec.  A pathspec of None or the
CLI's literal "null" counts as unset.  The artifact read is the trainer `Result` stored by the
training flow (`data.result`); its `.checkpoint` is returned.
"""
from __future__ import annotations

from .flowspec import current
from .registry import Run, Task


def _named(spec) -> bool:
    return spec is not None and spec != "null"


def _triggering_run():
    try:
        return current.trigger.run  # AttributeError: not event-triggered
    except AttributeError:
        return None


def upstream_checkpoint(task_spec=None, run_spec=None, use_trigger: bool = False, required: bool = True):
    """Checkpoint of the upstream training run; None when nothing names one and not `required`."""
    source = _triggering_run() if use_trigger else None
    if source is None and _named(task_spec):
        source = Task(task_spec)
    if source is None and _named(run_spec):
        source = Run(run_spec)
    if source is not None:
        return source.data.result.checkpoint
    if required:
        raise ValueError("If this run is not being triggered by RayTorchTrain, you must specify an upstream run or task id.")
    return None
