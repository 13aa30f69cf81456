from .gpt2 import GPT2, GPT2Config  # noqa: F401
from .layers import Dropout, Embedding, FusedReLU, LayerNorm, Linear, RMSNorm  # noqa: F401
from .mlp import NeuralNetwork  # noqa: F401
from .llama import Llama, LlamaConfig  # noqa: F401
from .resnet import ResNet18  # noqa: F401
