"""Linear layers on the native MFMA GEMMs, with fused epilogues.

* `linear(x, w, b, act, residual)` - bf16 activations (fp32 master params, bf16 shadows):
  forward = one GEMM with bias/ReLU/residual fused in the epilogue; backward = dgrad + wgrad
  GEMMs (fp32 weight gradient) + a deterministic bias-gradient column reduce.
* `fused_mlp(x, w_fc, b_fc, w_proj, b_proj, residual)` - the transformer MLP: the c_fc GEMM
  writes both the GELU output and its pre-activation, and in backward the c_proj dgrad GEMM
  applies GELU' in its epilogue (no separate GELU kernels in either direction).
* fp32 activations take the exact-f32 MFMA path (`gemm_f32`): the reference toy MLP.

On CPU every op is its PyTorch reference implementation (same math, autograd by torch).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import gemm as G
from ._ext import gpu_ext
from .gradbuf import grad_target
from .shadow import kmajor_image, kmajor_prefetch, kmajor_wanted, shadow_of


def _relu_mask_bwd(dy: torch.Tensor, y: torch.Tensor, p: float = 0.0) -> torch.Tensor:
    """dx = dy * (y > 0) (/ (1 - p): the output of a fused ReLU + inverted dropout is positive
    exactly where the unit was kept and active) on the native elementwise kernel."""
    dx = torch.empty_like(dy)
    gpu_ext().relu_dropout(y, None, dy, dx, float(p), 0, 0, 2 if p > 0.0 else 1)
    return dx


class _LinearBF16(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, residual, relu: bool):
        K = x.shape[-1]
        x2 = x.reshape(-1, K)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        ws = shadow_of(w)
        res2 = residual.reshape(-1, w.shape[0]) if residual is not None else None
        y = G.linear_fwd(x2, ws, bias=b, act=G.ACT_RELU if relu else G.ACT_NONE, residual=res2)
        # the input gradient's K-major weight image, built on a side stream under the forward
        ctx.kimg = ctx.needs_input_grad[0] and kmajor_wanted(w, x2.shape[0])
        if ctx.kimg:
            kmajor_prefetch(w)
        ctx.save_for_backward(x2, ws, y if relu else None)
        ctx.relu = relu
        ctx.has_b = b is not None
        ctx.has_res = residual is not None
        ctx.in_shape = x.shape
        ctx.params = (w, b)
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, ws, y = ctx.saved_tensors
        N = ws.shape[0]
        dy2 = dy.reshape(-1, N)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dpre = _relu_mask_bwd(dy2, y) if ctx.relu else dy2
        w, b = ctx.params
        dx = (G.linear_dgrad(dpre, ws, w_kmajor=kmajor_image(w) if ctx.kimg else None).view(ctx.in_shape)
              if ctx.needs_input_grad[0] else None)
        dw = G.linear_wgrad(dpre, x2, out=grad_target(w)) if ctx.needs_input_grad[1] else None
        db = G.colsum(dpre, out=grad_target(b)) if ctx.has_b and ctx.needs_input_grad[2] else None
        dres = dy if ctx.has_res else None
        return dx, dw, db, dres, None


class _LinearF32(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, relu: bool, drop=None):
        K = x.shape[-1]
        x2 = x.reshape(-1, K).contiguous()
        M, N = x2.shape[0], w.shape[0]
        y = torch.empty((M, N), dtype=torch.float32, device=x.device)
        G.gemm_f32(x2, w, y, M, N, K, K, 1, 1, K, N, bias=b, act=G.ACT_RELU if relu else G.ACT_NONE, dropout=drop)
        ctx.save_for_backward(x2, w, y if relu else None)
        ctx.relu = relu
        ctx.p = drop[0] if drop is not None else 0.0
        ctx.has_b = b is not None
        ctx.in_shape = x.shape
        ctx.bias = b
        return y.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, w, y = ctx.saved_tensors
        N, K = w.shape
        M = x2.shape[0]
        dy2 = dy.reshape(-1, N).contiguous()
        dpre = _relu_mask_bwd(dy2, y, ctx.p) if ctx.relu else dy2
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty((M, K), dtype=torch.float32, device=dy.device)
            G.gemm_f32(dpre, w, dx, M, K, N, N, 1, K, 1, K)
            dx = dx.view(ctx.in_shape)
        if ctx.needs_input_grad[1]:
            dw = grad_target(w)
            if dw is None:
                dw = torch.empty((N, K), dtype=torch.float32, device=dy.device)
            G.gemm_f32(dpre, x2, dw, N, K, M, 1, N, K, 1, K)
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = G.colsum(dpre, out=grad_target(ctx.bias))
        return dx, dw, db, None, None


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None, relu: bool = False,
           residual: torch.Tensor | None = None, dropout: float = 0.0, stream=None) -> torch.Tensor:
    """y = act(x w^T + b) (+ residual); dropout > 0 (training) applies inverted dropout after
    the ReLU - fused into the fp32 GEMM's epilogue, the Philox stream `stream` (default:
    ops.random.default_stream()) consumed exactly like a separate `ops.dropout` call."""
    if not x.is_cuda:
        y = F.linear(x, w.to(x.dtype), None if b is None else b.to(x.dtype))
        if relu:
            y = torch.relu(y)
        if dropout > 0.0:
            y = F.dropout(y, dropout, True)
        if residual is not None:
            y = y + residual
        return y
    if x.dtype == torch.float32:
        drop = None
        if dropout > 0.0 and relu and residual is None:
            from .random import default_stream

            st = stream or default_stream()
            n = x.numel() // x.shape[-1] * w.shape[0]
            seed, offset = st.reserve(n)
            drop = (dropout, seed, offset, st.device_base())
        y = _LinearF32.apply(x, w, b, relu, drop)
        if dropout > 0.0 and drop is None:
            from .dropout import dropout as _dropout

            y = _dropout(y, dropout, True, stream)
        return y + residual if residual is not None else y
    y = _LinearBF16.apply(x, w, b, residual if dropout == 0.0 else None, relu)
    if dropout > 0.0:
        from .dropout import dropout as _dropout

        y = _dropout(y, dropout, True, stream)
        if residual is not None:
            y = y + residual
    return y


# 1: the c_fc forward stores gelu'(pre) and the backward multiplies by it (act 5 / 6);
# 0 (default): it stores the pre-activation and the backward evaluates gelu' (act 2 / 3).
# Measured neutral on GPT-2-small (profiles/gelu_save_grad_ab.txt): the dgrad epilogue is not
# bound by its two transcendentals, so the numerics stay on the original pair.
_GELU_SAVE_GRAD = os.environ.get("RTDC_GELU_SAVE_GRAD", "0") == "1"
class _FusedMLP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w_fc, b_fc, w_proj, b_proj, residual):
        C = x.shape[-1]
        x2 = x.reshape(-1, C)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        M = x2.shape[0]
        H = w_fc.shape[0]
        wfs, wps = shadow_of(w_fc), shadow_of(w_proj)
        # side output: the pre-activation (or gelu'(pre) with RTDC_GELU_SAVE_GRAD=1)
        pre = torch.empty((M, H), dtype=torch.bfloat16, device=x.device)
        g = G.linear_fwd(x2, wfs, bias=b_fc, act=G.ACT_GELU_SAVE_GRAD if _GELU_SAVE_GRAD else G.ACT_GELU,
                         aux_out=pre)
        res2 = residual.reshape(-1, C) if residual is not None else None
        y = G.linear_fwd(g, wps, bias=b_proj, residual=res2)
        # both input gradients on K-major weight images (ops/shadow.py), built under the forward:
        # c_proj's (dpre = dy . W_proj with GELU' and the c_fc bias column sums) and c_fc's
        ctx.kimg = (ctx.needs_input_grad[0] or ctx.needs_input_grad[1]) and kmajor_wanted(w_proj, M)
        if ctx.kimg:
            kmajor_prefetch(w_proj)
            if ctx.needs_input_grad[0]:
                kmajor_prefetch(w_fc)
        ctx.save_for_backward(x2, wfs, wps, pre, g)
        ctx.has_res = residual is not None
        ctx.in_shape = x.shape
        ctx.params = (w_fc, b_fc, w_proj, b_proj)
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, wfs, wps, pre, g = ctx.saved_tensors
        C = x2.shape[1]
        dy2 = dy.reshape(-1, C)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        w_fc, b_fc, w_proj, b_proj = ctx.params
        dw_proj = G.linear_wgrad(dy2, g, out=grad_target(w_proj))
        db_proj = G.colsum(dy2, out=grad_target(b_proj))
        # c_fc's bias gradient = column sums of dpre, reduced in the dgrad GEMM's epilogue
        db_fc = grad_target(b_fc)
        if db_fc is None and b_fc is not None:
            db_fc = torch.empty(b_fc.shape, dtype=torch.float32, device=dy2.device)
        act = G.ACT_MUL if _GELU_SAVE_GRAD else G.ACT_GELU_BWD
        dpre = G.linear_dgrad(dy2, wps, act_bwd=act, aux_in=pre, colsum_out=db_fc,
                              w_kmajor=kmajor_image(w_proj) if ctx.kimg else None)
        dw_fc = G.linear_wgrad(dpre, x2, out=grad_target(w_fc))
        dx = G.linear_dgrad(dpre, wfs, w_kmajor=kmajor_image(w_fc) if ctx.kimg else None).view(ctx.in_shape)
        return dx, dw_fc, db_fc, dw_proj, db_proj, (dy if ctx.has_res else None)


def gelu_tanh_ref(x):
    return F.gelu(x, approximate="tanh")


def fused_mlp(x, w_fc, b_fc, w_proj, b_proj, residual=None):
    if not x.is_cuda:
        h = gelu_tanh_ref(F.linear(x, w_fc.to(x.dtype), b_fc.to(x.dtype)))
        y = F.linear(h, w_proj.to(x.dtype), b_proj.to(x.dtype))
        return y + residual if residual is not None else y
    return _FusedMLP.apply(x, w_fc, b_fc, w_proj, b_proj, residual)
