"""LayerNorm / RMSNorm on the native wave64 row kernels (bf16 activations, fp32 master params)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import gemm as G
from ._ext import gpu_ext
from .shadow import shadow_of


def _bwd_waves(M: int) -> int:
    # up to 4096 waves (4 blocks of 4 waves per CU) for latency hiding; the kernel combines
    # each block's 4 waves, so the partial workspace is (waves / 4) rows
    return max(4, min(4096, (M + 3) // 4 * 4))


def _bwd_ws_elems(nw: int, D: int) -> int:
    return (2 * (nw // 4) + 2 * 64) * D


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        D = x.shape[-1]
        xc = x.contiguous()
        M = xc.numel() // D
        y = torch.empty_like(xc)
        mean = torch.empty(M, dtype=torch.float32, device=x.device)
        rstd = torch.empty(M, dtype=torch.float32, device=x.device)
        ws, bs = shadow_of(w), shadow_of(b)
        gpu_ext().layernorm_fwd(xc, ws, bs, y, mean, rstd, eps)
        ctx.save_for_backward(xc, ws, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, ws, mean, rstd = ctx.saved_tensors
        D = xc.shape[-1]
        M = xc.numel() // D
        nw = _bwd_waves(M)
        wsp = G.workspace(xc.device, _bwd_ws_elems(nw, D), "ln_bwd")
        dx = torch.empty_like(xc)
        dg = torch.empty(D, dtype=torch.float32, device=xc.device)
        db = torch.empty(D, dtype=torch.float32, device=xc.device)
        gpu_ext().layernorm_bwd(dy.contiguous(), xc, ws, mean, rstd, None, dx, wsp, dg, db, nw, False)
        return dx, dg, db, None


class _RMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps):
        D = x.shape[-1]
        xc = x.contiguous()
        M = xc.numel() // D
        y = torch.empty_like(xc)
        rstd = torch.empty(M, dtype=torch.float32, device=x.device)
        ws = shadow_of(w)
        gpu_ext().rmsnorm_fwd(xc, ws, y, rstd, eps)
        ctx.save_for_backward(xc, ws, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, ws, rstd = ctx.saved_tensors
        D = xc.shape[-1]
        M = xc.numel() // D
        nw = _bwd_waves(M)
        wsp = G.workspace(xc.device, _bwd_ws_elems(nw, D), "rms_bwd")
        dx = torch.empty_like(xc)
        dg = torch.empty(D, dtype=torch.float32, device=xc.device)
        gpu_ext().rmsnorm_bwd(dy.contiguous(), xc, ws, rstd, None, dx, wsp, dg, nw, False)
        return dx, dg, None


def layer_norm(x, w, b, eps=1e-5):
    if not x.is_cuda or x.dtype != torch.bfloat16:
        return F.layer_norm(x, (x.shape[-1],), w.to(x.dtype), b.to(x.dtype), eps)
    return _LayerNorm.apply(x, w, b, eps)


def rms_norm(x, w, eps=1e-5):
    if not x.is_cuda or x.dtype != torch.bfloat16:
        xf = x.float()
        y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
        return (y * w.float()).to(x.dtype)
    return _RMSNorm.apply(x, w, eps)
