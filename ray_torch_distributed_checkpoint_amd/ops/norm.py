"""LayerNorm / RMSNorm on the native wave64 row kernels (bf16 activations, fp32 master params)."""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import gemm as G
from ._ext import gpu_ext, require_dtype
from .gradbuf import grad_target
from .shadow import shadow_of


_BWD_WAVES = int(os.environ.get("RTDC_NORM_BWD_WAVES", "4096"))


def _bwd_waves(M: int) -> int:
    # up to 4096 waves (4 blocks of 4 waves per CU) for latency hiding; the kernel combines
    # each block's 4 waves, so the partial workspace is (waves / 4) rows
    return max(4, min(_BWD_WAVES, (M + 3) // 4 * 4))


def _bwd_ws_elems(nw: int, D: int, nz: int = 3) -> int:
    # nz reductions (dgamma, dbeta, colsum(dx)): [nz][nw/4][D] partials + nz x [64][D] rows
    return nz * (nw // 4 + 64) * D


class _LayerNorm(torch.autograd.Function):
    """y = LN(x).  With passthrough=True also returns x itself (the residual stream): its
    gradient arrives as a second output gradient and is added inside the backward kernel
    (dres) instead of by a separate autograd add."""

    @staticmethod
    def forward(ctx, x, w, b, eps, passthrough=False, sum_param=None):
        ctx.set_materialize_grads(False)
        D = x.shape[-1]
        xc = x.contiguous()
        M = xc.numel() // D
        y = torch.empty_like(xc)
        mean = torch.empty(M, dtype=torch.float32, device=x.device)
        rstd = torch.empty(M, dtype=torch.float32, device=x.device)
        ws, bs = shadow_of(w), shadow_of(b)
        gpu_ext().layernorm_fwd(xc, ws, bs, y, mean, rstd, eps)
        ctx.save_for_backward(xc, ws, mean, rstd)
        ctx.params = (w, b)
        ctx.sum_param = sum_param
        return (y, xc) if passthrough else y

    @staticmethod
    def backward(ctx, dy, dpass=None):
        xc, ws, mean, rstd = ctx.saved_tensors
        if dy is None:
            dy = torch.zeros_like(xc)
        D = xc.shape[-1]
        M = xc.numel() // D
        nw = _bwd_waves(M)
        wsp = G.workspace(xc.device, _bwd_ws_elems(nw, D), "ln_bwd")
        dx = torch.empty_like(xc)
        w, b = ctx.params
        dg, db = grad_target(w), grad_target(b)
        if dg is None or db is None:
            dgb = torch.empty((2, D), dtype=torch.float32, device=xc.device)
            dg = dgb[0] if dg is None else dg
            db = dgb[1] if db is None else db
        dres = dpass.contiguous() if dpass is not None else None
        # dx is the residual-stream gradient: its column sums are the bias gradient of the
        # residual projection that produced x (sum_param: attention / MLP c_proj bias).  They
        # are reduced by this kernel on the way out - straight into that bias's slot of the
        # flat gradient buffer when it has one - and offered to the projection's colsum(),
        # which then returns them as the bias gradient without touching dx again.
        dxsum = None
        if ctx.sum_param is not None:
            dxsum = grad_target(ctx.sum_param)
            if dxsum is None:
                dxsum = torch.empty(D, dtype=torch.float32, device=xc.device)
        outs = [dg, db] + ([dxsum] if dxsum is not None else [])
        if all(G._deferrable(o) for o in outs):
            # partial rows into a buffer of their own, reduced with the deferred window (gemm.py)
            part = torch.empty(len(outs) * (nw // 4 + 64) * D, dtype=torch.float32, device=xc.device)
            nblk = gpu_ext().layernorm_bwd(dy.contiguous(), xc, ws, mean, rstd, dres, dx, part, dg, db, dxsum, nw,
                                           False, True)
            rows = part[: len(outs) * nblk * D].view(len(outs), nblk * D)
            done = [G._WG.add_job(rows[z], nblk, D, o, False) for z, o in enumerate(outs)]
            if not all(done):
                if any(done):
                    G.flush_wgrads()
                gpu_ext().colsum_multi([rows[z] for z, d in enumerate(done) if not d],
                                       [o for o, d in zip(outs, done) if not d],
                                       [nblk] * done.count(False), [D] * done.count(False), [0] * done.count(False))
        else:
            gpu_ext().layernorm_bwd(dy.contiguous(), xc, ws, mean, rstd, dres, dx, wsp, dg, db, dxsum, nw, False,
                                    False)
        if dxsum is not None:
            G.offer_colsum(dx, dxsum)
        return dx, dg, db, None, None, None


class _RMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps, passthrough=False):
        ctx.set_materialize_grads(False)
        D = x.shape[-1]
        xc = x.contiguous()
        M = xc.numel() // D
        y = torch.empty_like(xc)
        rstd = torch.empty(M, dtype=torch.float32, device=x.device)
        ws = shadow_of(w)
        gpu_ext().rmsnorm_fwd(xc, ws, y, rstd, eps)
        ctx.save_for_backward(xc, ws, rstd)
        ctx.w = w
        return (y, xc) if passthrough else y

    @staticmethod
    def backward(ctx, dy, dpass=None):
        xc, ws, rstd = ctx.saved_tensors
        if dy is None:
            dy = torch.zeros_like(xc)
        D = xc.shape[-1]
        M = xc.numel() // D
        nw = _bwd_waves(M)
        wsp = G.workspace(xc.device, _bwd_ws_elems(nw, D), "rms_bwd")
        dx = torch.empty_like(xc)
        dg = grad_target(ctx.w)
        if dg is None:
            dg = torch.empty(D, dtype=torch.float32, device=xc.device)
        dres = dpass.contiguous() if dpass is not None else None
        gpu_ext().rmsnorm_bwd(dy.contiguous(), xc, ws, rstd, dres, dx, wsp, dg, None, nw, False)
        return dx, dg, None, None


def layer_norm(x, w, b, eps=1e-5, passthrough=False, grad_sum_into=None):
    """LayerNorm over the last axis; passthrough=True returns (y, x) with the residual-stream
    gradient fused into the backward kernel.  grad_sum_into: the bias of the projection that
    produced x; its gradient (= column sums of dx) is then reduced by the backward kernel."""
    if x.is_cuda:
        require_dtype(x, "layer_norm")
    else:
        y = F.layer_norm(x, (x.shape[-1],), w.to(x.dtype), b.to(x.dtype), eps)
        return (y, x) if passthrough else y
    return _LayerNorm.apply(x, w, b, eps, passthrough, grad_sum_into)


def rms_norm(x, w, eps=1e-5, passthrough=False):
    if x.is_cuda:
        require_dtype(x, "rms_norm")
    else:
        xf = x.float()
        y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
        y = (y * w.float()).to(x.dtype)
        return (y, x) if passthrough else y
    return _RMSNorm.apply(x, w, eps, passthrough)
