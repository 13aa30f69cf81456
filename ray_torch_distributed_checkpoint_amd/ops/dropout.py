"""Dropout on the native Philox kernel; the mask is regenerated in backward from (seed, offset)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ._ext import gpu_ext
from .random import PhiloxStream, default_stream


class _Dropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed, offset, base):
        xc = x.contiguous()
        y = torch.empty_like(xc)
        gpu_ext().dropout(xc, y, p, seed, offset, base)
        ctx.p, ctx.seed, ctx.offset, ctx.base = p, seed, offset, base
        return y

    @staticmethod
    def backward(ctx, dy):
        dyc = dy.contiguous()
        dx = torch.empty_like(dyc)
        gpu_ext().dropout(dyc, dx, ctx.p, ctx.seed, ctx.offset, ctx.base)
        return dx, None, None, None, None


def dropout(x: torch.Tensor, p: float, training: bool = True, stream: PhiloxStream | None = None):
    if not training or p == 0.0:
        return x
    if not x.is_cuda:
        return F.dropout(x, p, training)
    st = stream or default_stream()
    seed, offset = st.reserve(x.numel())
    return _Dropout.apply(x, p, seed, offset, st.device_base())
