"""MI355X-native ops: hand-written gfx950 HIP kernels behind autograd-compatible functions.

GPU tensors always run the native kernels (the extension is mandatory on a GPU box); CPU
tensors run the PyTorch reference implementation of the same op (used by the CPU test-suite
and gloo multi-process tests).
"""
from ._ext import available as native_available, ext  # noqa: F401
from .attention import causal_attention  # noqa: F401
from .dropout import dropout  # noqa: F401
from .embedding import embedding  # noqa: F401
from .linear import fused_mlp, linear  # noqa: F401
from .norm import layer_norm, rms_norm  # noqa: F401
from .random import PhiloxStream, default_stream, manual_seed  # noqa: F401
from .shadow import shadow_of  # noqa: F401
from .xent import cross_entropy, lm_head_cross_entropy, xent_metrics  # noqa: F401
