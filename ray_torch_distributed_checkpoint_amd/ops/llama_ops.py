"""Rotary embedding (on the packed QKV buffer) and SwiGLU on the native kernels."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import gemm as G
from ._ext import gpu_ext, require_dtype
from .gradbuf import grad_target
from .shadow import shadow_of

_tables: dict = {}


def rope_tables(T: int, Dh: int, theta: float, device) -> tuple[torch.Tensor, torch.Tensor]:
    """Host-precomputed cos/sin [T, Dh/2] (fp32), cached per device."""
    key = (T, Dh, float(theta), str(device))
    t = _tables.get(key)
    if t is None:
        inv = 1.0 / (theta ** (torch.arange(0, Dh, 2, dtype=torch.float64) / Dh))
        ang = torch.arange(T, dtype=torch.float64)[:, None] * inv[None, :]
        t = (ang.cos().float().to(device).contiguous(), ang.sin().float().to(device).contiguous())
        _tables[key] = t
    return t


def rope_ref(qkv: torch.Tensor, H: int, Hkv: int, theta: float) -> torch.Tensor:
    B, T, W = qkv.shape
    Dh = W // (H + 2 * Hkv)
    cos, sin = rope_tables(T, Dh, theta, qkv.device)
    x = qkv.view(B, T, H + 2 * Hkv, Dh)
    rot = x[:, :, : H + Hkv].float()
    x1, x2 = rot[..., : Dh // 2], rot[..., Dh // 2:]
    c, s = cos[None, :, None, :], sin[None, :, None, :]
    out = torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1).to(qkv.dtype)
    return torch.cat([out, x[:, :, H + Hkv:]], dim=2).view(B, T, W)


class _RoPE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, H, Hkv, theta):
        B, T, W = qkv.shape
        Dh = W // (H + 2 * Hkv)
        cos, sin = rope_tables(T, Dh, theta, qkv.device)
        x = qkv.contiguous()
        y = torch.empty_like(x)
        gpu_ext().rope(x, y, cos, sin, T, H + Hkv, H + 2 * Hkv, Dh, False)
        ctx.meta = (T, H, Hkv, Dh, cos, sin)
        return y

    @staticmethod
    def backward(ctx, dy):
        T, H, Hkv, Dh, cos, sin = ctx.meta
        d = dy.contiguous()
        dx = torch.empty_like(d)
        gpu_ext().rope(d, dx, cos, sin, T, H + Hkv, H + 2 * Hkv, Dh, True)
        return dx, None, None, None


def apply_rope(qkv: torch.Tensor, n_head: int, n_kv_head: int, theta: float = 500000.0) -> torch.Tensor:
    if qkv.is_cuda:
        require_dtype(qkv, "apply_rope")
    else:
        return rope_ref(qkv, n_head, n_kv_head, theta)
    return _RoPE.apply(qkv, n_head, n_kv_head, theta)


class _SwiGLUMLP(torch.autograd.Function):
    """y = (silu(x W1^T) * (x W3^T)) W2^T (+ residual), with W1|W3 as ONE [2F, C] GEMM."""

    @staticmethod
    def forward(ctx, x, w13, w2, residual):
        C = x.shape[-1]
        x2 = x.reshape(-1, C)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        w13s, w2s = shadow_of(w13), shadow_of(w2)
        F2 = w13s.shape[0]
        gu = G.linear_fwd(x2, w13s)  # [M, 2F]
        h = torch.empty((x2.shape[0], F2 // 2), dtype=torch.bfloat16, device=x.device)
        gpu_ext().swiglu_fwd(gu, h)
        res2 = residual.reshape(-1, C) if residual is not None else None
        y = G.linear_fwd(h, w2s, residual=res2)
        ctx.save_for_backward(x2, w13s, w2s, gu, h)
        ctx.params = (w13, w2)
        ctx.has_res = residual is not None
        ctx.in_shape = x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w13s, w2s, gu, h = ctx.saved_tensors
        C = x2.shape[1]
        dy2 = dy.reshape(-1, C)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        w13, w2 = ctx.params
        dw2 = G.linear_wgrad(dy2, h, out=grad_target(w2))
        dh = G.linear_dgrad(dy2, w2s)
        dgu = torch.empty_like(gu)
        gpu_ext().swiglu_bwd(gu, dh, dgu)
        dw13 = G.linear_wgrad(dgu, x2, out=grad_target(w13))
        dx = G.linear_dgrad(dgu, w13s).view(ctx.in_shape)
        return dx, dw13, dw2, (dy if ctx.has_res else None)


def swiglu_mlp(x, w13, w2, residual=None):
    if x.is_cuda:
        require_dtype(x, "swiglu_mlp")
    else:
        gu = F.linear(x, w13.to(x.dtype))
        g, u = gu.chunk(2, dim=-1)
        y = F.linear(F.silu(g) * u, w2.to(x.dtype))
        return y + residual if residual is not None else y
    return _SwiGLUMLP.apply(x, w13, w2, residual)
