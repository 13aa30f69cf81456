"""nn.Module wrappers over the native ops.  Parameters are fp32 masters; GPU compute is bf16
(or exact fp32 for fp32 activations) on the hand-written gfx950 kernels."""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .. import ops


class Linear(nn.Module):
    """y = act(x W^T + b); `relu=True` fuses the ReLU into the GEMM epilogue."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True, relu: bool = False,
                 dropout: float = 0.0):
        super().__init__()
        self.in_features, self.out_features, self.relu = in_features, out_features, relu
        self.dropout = dropout  # inverted dropout after the ReLU, fused into the GEMM epilogue
        self.weight = nn.Parameter(torch.empty(out_features, in_features))
        self.bias = nn.Parameter(torch.empty(out_features)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        # nn.Linear's default init
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            bound = 1 / math.sqrt(self.in_features) if self.in_features > 0 else 0
            nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x, residual=None):
        return ops.linear(x, self.weight, self.bias, relu=self.relu, residual=residual,
                          dropout=self.dropout if self.training else 0.0)

    def extra_repr(self):
        r = f"in_features={self.in_features}, out_features={self.out_features}, bias={self.bias is not None}, " \
            f"fused_relu={self.relu}"
        return r + (f", fused_dropout={self.dropout}" if self.dropout else "")


class FusedReLU(nn.Module):
    """Placeholder keeping nn.Sequential indices (and state_dict keys) of a ReLU that was
    fused into the preceding Linear's epilogue."""

    def forward(self, x):
        return x

    def extra_repr(self):
        return "fused into previous Linear"


class FusedDropout(nn.Module):
    """Placeholder keeping nn.Sequential indices of a Dropout fused into the preceding Linear's
    epilogue (`Linear(..., relu=True, dropout=p)`)."""

    def __init__(self, p: float = 0.5):
        super().__init__()
        self.p = p

    def forward(self, x):
        return x

    def extra_repr(self):
        return f"p={self.p}, fused into previous Linear"


class Dropout(nn.Module):
    def __init__(self, p: float = 0.5):
        super().__init__()
        self.p = p

    def forward(self, x):
        return ops.dropout(x, self.p, self.training)

    def extra_repr(self):
        return f"p={self.p}"


class LayerNorm(nn.Module):
    def __init__(self, dim: int, eps: float = 1e-5):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim))
        self.bias = nn.Parameter(torch.zeros(dim))

    def forward(self, x, passthrough: bool = False, grad_sum_into=None):
        """passthrough=True -> (LN(x), x): use the second output as the residual so its
        gradient is folded into the norm's backward kernel.  grad_sum_into: bias of the
        projection that produced x, whose gradient the backward kernel then reduces."""
        return ops.layer_norm(x, self.weight, self.bias, self.eps, passthrough=passthrough,
                              grad_sum_into=grad_sum_into)


class RMSNorm(nn.Module):
    def __init__(self, dim: int, eps: float = 1e-5):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim))

    def forward(self, x, passthrough: bool = False):
        return ops.rms_norm(x, self.weight, self.eps, passthrough=passthrough)


class Embedding(nn.Module):
    def __init__(self, num: int, dim: int):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(num, dim))
        nn.init.normal_(self.weight, std=0.02)
