"""Metaflow-compatible flow runner, run registry, cards (replaces Metaflow + metaflow-ray for the
reference's train/eval flows on one MI355X node)."""
from .cards import Artifact, Image, Markdown, Table  # noqa: F401
from .flowspec import (FlowSpec, Parameter, card, conda, current, environment, gpu_profile,  # noqa: F401
                       kubernetes, metaflow_ray, pypi, resources, retry, schedule, step, trigger_on_finish)
from .registry import Flow, Run, Step, Task, namespace  # noqa: F401
from .upstream import upstream_checkpoint  # noqa: F401
