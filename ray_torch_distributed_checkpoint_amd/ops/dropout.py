"""Dropout on the native Philox kernel; the mask is regenerated in backward from (seed, offset)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ._ext import gpu_ext
from .random import PhiloxStream, default_stream


class _Dropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed, offset):
        xc = x.contiguous()
        y = torch.empty_like(xc)
        gpu_ext().dropout(xc, y, p, seed, offset)
        ctx.p, ctx.seed, ctx.offset = p, seed, offset
        return y

    @staticmethod
    def backward(ctx, dy):
        dyc = dy.contiguous()
        dx = torch.empty_like(dyc)
        gpu_ext().dropout(dyc, dx, ctx.p, ctx.seed, ctx.offset)
        return dx, None, None, None


def dropout(x: torch.Tensor, p: float, training: bool = True, stream: PhiloxStream | None = None):
    if not training or p == 0.0:
        return x
    if not x.is_cuda:
        return F.dropout(x, p, training)
    seed, offset = (stream or default_stream()).reserve(x.numel())
    return _Dropout.apply(x, p, seed, offset)
