from .gpt2 import GPT2, GPT2Config  # noqa: F401
from .layers import Dropout, Embedding, FusedReLU, LayerNorm, Linear, RMSNorm  # noqa: F401
from .mlp import NeuralNetwork  # noqa: F401
