"""The reference toy model (R/my_ray_module.py:94-112), same module tree and state_dict keys
(`linear_relu_stack.{0,3,6}.{weight,bias}`), on native kernels: each Linear+ReLU pair is one
exact-f32 MFMA GEMM with the ReLU in its epilogue (the ReLU slot keeps its index as a
`FusedReLU` placeholder), and the Philox dropout mask is drawn in the same epilogue
(`FusedDropout` placeholder).  The final ReLU on the logits is kept
(reference quirk)."""
from __future__ import annotations

import torch.nn as nn

from .layers import FusedDropout, FusedReLU, Linear


class NeuralNetwork(nn.Module):
    def __init__(self, dropout: float = 0.25):
        super().__init__()
        self.flatten = nn.Flatten()
        # Linear + ReLU + Dropout is ONE fp32 MFMA GEMM: bias, ReLU and the Philox mask in its
        # epilogue (the ReLU / Dropout slots keep their indices as placeholders)
        self.linear_relu_stack = nn.Sequential(
            Linear(28 * 28, 512, relu=True, dropout=dropout),
            FusedReLU(),
            FusedDropout(dropout),
            Linear(512, 512, relu=True, dropout=dropout),
            FusedReLU(),
            FusedDropout(dropout),
            Linear(512, 10, relu=True),
            FusedReLU(),
        )

    def forward(self, x):
        x = self.flatten(x)
        return self.linear_relu_stack(x)
